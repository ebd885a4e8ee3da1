"""Multi-agent ensemble evaluator — the reference's combiner scripts on edgellm.

    python -m edgellm.cli.combine --config config.yaml [--max_new_tokens 200 ...]            # C4/C7 (fp)
    python -m edgellm.cli.combine --config config.yaml --quant llm_int8                      # C5/C6 (bnb-style INT8)
    python -m edgellm.cli.combine --config config.yaml --quant w8a8_smoothquant --merge vote  # north star

Same YAML keys / 13 CLI flags / log lines as Code/Base Models/combine_model_fp_updated.py:138-232
(and Code/Quantised Models/combiner_quant_updated.py).  Agents run concurrently on separate
GPUs; the refiner merges (or a majority vote).  Per-sample metrics: ROUGE-1/2/L, BERTScore,
BLEU, cosine, confidence (scored with the refiner, as combine_model_fp_updated.py:208; a vote
merge loads no refiner, so there the FIRST QA agent scores it — every metrics row names its scorer
in ``confidence_scorer``: do not compare vote-mode confidence with refiner-scored runs), combo TPS =
mean of the QA agents' TPS.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import List, Optional

import torch

from ..config import add_reference_args, apply_overrides, load_config, RunConfig
from ..data import load_qa
from ..engine import Generator, SamplingParams
from ..eval import EfficiencyMeter, Embedder, MetricSuite, ProgressLog, Results
from ..eval.metrics import confidence_scores
from ..models.registry import load_model
from ..orchestrator import Agent, Orchestrator, RefineMerge, VoteMerge
from ..parallel.split import agent_devices, split_model
from ..utils.log import format_efficiency_report, format_final_report, get_logger
from .common import (add_runtime_args, build_generator, build_pp_engine, pick_devices, pop_runtime, pp_launch,
                     resolve_runtime)

logger = get_logger("combine")


def build_embedder(name: Optional[str], base_dir: Optional[str], device) -> Embedder:
    from ..models.bert import BertEncoder, load_bert
    from ..models.hf import resolve_model_dir
    from ..utils.tokenizer import load_tokenizer
    path = resolve_model_dir(name, base_dir) if name else None
    if path:
        enc = load_bert(path, device=device)
        return Embedder(enc, load_tokenizer(path), device)
    logger.warning(f"No embedder checkpoint for '{name}': random-init MiniLM-L6 encoder (cosine/BERTScore are synthetic)")
    torch.manual_seed(0)
    enc = BertEncoder(device=device).eval()
    from ..utils.tokenizer import ByteTokenizer
    return Embedder(enc, ByteTokenizer(enc.cfg.vocab_size), device)


def make_agent(name: str, model_id: str, precision: str, quant: str, device, sampling: SamplingParams, rt: dict,
               cpu_prompt: bool = False, gpus=None, launch=None, tag: int = 0) -> Agent:
    """One agent: the model on ``device``, or split layer-wise over its GPU group (``gpus``, the
    YAML ``agents[].gpus``; else ``pp_size`` devices from ``device``) — the reference's
    ``device_map="auto"`` placement (combine_model_fp_updated.py:40).  Under torchrun
    (``launch``) this rank's pipeline stage behind a PipelineGenerator (parallel/pp_engine.py)."""
    if launch is not None:
        eng, tok, source, bounds = build_pp_engine(model_id, precision, quant, rt, launch, tag,
                                                   max_batch=int(rt.get("batch_size") or 1), gpus=gpus)
        if eng.member:
            logger.info(f"{name}: {source} pipelined over {len(eng.ranks)} ranks {eng.ranks} at layers {bounds} "
                        f"({quant})")
        return Agent(name, eng, tok, sampling, cpu_prompt)
    devs = agent_devices(gpus, torch.device(device), int(rt.get("pp_size") or 1))
    model, tok, source = load_model(model_id, precision, quant, devs[0], rt.get("base_model_path"))
    if len(devs) > 1:
        model = split_model(model, devs)
        logger.info(f"{name}: {source} split over {[str(d) for d in devs]} at layers {model.bounds} ({quant})")
    else:
        logger.info(f"{name}: {source} on {devs[0]} ({quant}, {str(model.dtype).replace('torch.', '')})")
    gen = build_generator(model, rt, max_batch=int(rt.get("batch_size") or 1))
    return Agent(name, gen, tok, sampling, cpu_prompt)


def run_ensemble(cfg: RunConfig, rt: dict, qa_specs, refiner_spec, cpu_variant: bool = False) -> dict:
    """qa_specs: (name, model, precision[, quant[, gpus]]) per QA agent."""
    rt = resolve_runtime(cfg, rt)
    quant = rt.get("quant") or cfg.quant.mode
    launch = pp_launch(rt)                        # torchrun: every model pipelined over the ranks
    devices = [launch[2]] if launch is not None else pick_devices(rt.get("devices"))
    s = cfg.sampling
    sampling = SamplingParams(s.max_new_tokens, s.temperature, s.top_k, s.top_p, s.repetition_penalty, s.do_sample)
    logger.info("Loading dataset...")
    rows = load_qa(cfg.dataset_name, cfg.dataset_split, cfg.dataset_path, rt.get("num_samples"))
    logger.info("Loading models...")
    agents = []
    for i, spec in enumerate(qa_specs):
        n, mid, prec = spec[:3]
        aq = spec[3] if len(spec) > 3 and spec[3] not in (None, "none") else quant
        gpus = spec[4] if len(spec) > 4 else None
        agents.append(make_agent(n, mid, prec, aq, devices[i % len(devices)], sampling, rt, cpu_variant, gpus,
                                 launch=launch, tag=i))
    merge_kind = rt.get("merge") or cfg.merge
    refiner = None
    if merge_kind == "refine" and refiner_spec is not None:      # (vote: no refiner model is loaded)
        rn, rid, rprec = refiner_spec
        refiner = make_agent(rn, rid, rprec, quant, devices[len(agents) % len(devices)], sampling, rt,
                             launch=launch, tag=len(agents))
    if launch is not None:
        from ..parallel.pp_engine import serve_workers, stop_workers
        if launch[0] != 0:                        # workers: serve the driver's commands until STOP
            serve_workers({a.generator.tag: a.generator for a in agents + ([refiner] if refiner else [])})
            return {}
        # no STOP on an exception: the driver's exit makes torchrun tear the workers down (a STOP
        # broadcast could meet a worker blocked inside a pipeline exchange)
        out = _ensemble_loop(cfg, rt, agents, refiner, merge_kind, rows, devices, cpu_variant)
        stop_workers(agents[0].generator)
        return out
    return _ensemble_loop(cfg, rt, agents, refiner, merge_kind, rows, devices, cpu_variant)


def _ensemble_loop(cfg, rt, agents, refiner, merge_kind, rows, devices, cpu_variant) -> dict:
    legacy = not rt.get("no_legacy_decode", False)
    if merge_kind == "vote":
        merge = VoteMerge()
    else:
        merge = RefineMerge(refiner, include_reference=not rt.get("no_reference_in_refiner", False),
                            legacy_decode=legacy)
    orch = Orchestrator(agents, merge, concurrent=not rt.get("serial", False), legacy_decode=legacy,
                        tps_includes_merger=cpu_variant)
    logger.info("Loading embedder model...")
    suite = MetricSuite(build_embedder(cfg.embedder_model, rt.get("base_model_path"), devices[0]))
    scorer = refiner or agents[0]
    scorer_name = "refiner" if refiner is not None else f"agent:{agents[0].name}"
    if refiner is None:
        logger.warning(f"merge=vote: confidence is scored with QA agent '{agents[0].name}' (no refiner is loaded); "
                       "the reference scores it with the refiner")
    progress = ProgressLog(rt.get("progress"))
    done = progress.done()
    results = Results()
    eff = EfficiencyMeter([a.device for a in agents] + ([refiner.device] if refiner else []))
    bs = max(1, int(rt.get("batch_size") or 1))
    # per-agent tokens/sec under both of the reference's definitions, per sample (a batch's rows share
    # its generate wall): generated-only (the combiners, combine_model_fp_updated.py:106-108) and
    # prompt + generated (the single-model scripts, Llama_bf16_updated.py:89-90)
    agent_tps = {a.name: {"gen": [], "all": []} for a in agents}
    logger.info("Starting evaluation loop..." + (f" ({bs} questions per batch)" if bs > 1 else ""))
    todo = [i for i in range(len(rows)) if i not in done]
    for i in done:
        results.add({k: done[i][k] for k in done[i] if k not in ("index",)})
    for j0 in range(0, len(todo), bs):
        idx = todo[j0:j0 + bs]
        qs, refs = [rows[i]["query"] for i in idx], [rows[i]["answer"] for i in idx]
        for q in qs:
            logger.info(f"Processing question: {q}")
        t0 = time.perf_counter()
        if bs == 1:
            outs = [orch.answer(qs[0], refs[0], seed=rt.get("seed", 0) + idx[0])]
        else:
            outs = orch.answer_batch(qs, refs, seed=rt.get("seed", 0) + idx[0])
        confs = [None] * len(outs)
        if bs > 1 and scorer is not None:          # one padded scorer pass per 32 answers
            try:
                confs = confidence_scores(scorer.generator.model, [scorer.tokenizer.encode(r.final) for r in outs])
            except Exception:
                confs = [None] * len(outs)
        for i, q, ref, res, conf in zip(idx, qs, refs, outs, confs):
            for name, ans in res.answers.items():
                logger.info(f"Answer from {name}: {ans[:100]}...")
                if cpu_variant:
                    logger.info(f"[Q{i + 1}] {name} TPS: {res.tps[name]:.2f} tokens/sec")
            logger.info(f"Refined response: {res.final[:100]}...")
            m = suite.score(res.final, ref, scorer.generator.model, scorer.tokenizer, tps=res.combo_tps,
                            confidence=conf)
            if m["rouge1"] == 0.0 and m["tps"] == 0.0:
                logger.error("Error in evaluation: metrics zeroed for this sample")
            results.add(m)
            progress.append(i, m)
            if rt.get("metrics_jsonl"):
                with open(rt["metrics_jsonl"], "a") as f:
                    f.write(json.dumps({"index": i, **m, "agent_tps": res.tps, "wall_s": res.wall_s,
                                        "confidence_scorer": scorer_name, "answers": res.answers,
                                        "final": res.final}) + "\n")
            if cpu_variant:
                logger.info(f"[Q{i + 1}] Total time: {res.wall_s:.2f} sec\n")
        for name, g in outs[0].results.items():
            if name in agent_tps and g.elapsed_s > 0:
                for toks, pl in zip(g.tokens, g.prompt_lens):
                    agent_tps[name]["gen"].append(len(toks) / g.elapsed_s)
                    agent_tps[name]["all"].append((len(toks) + pl) / g.elapsed_s)
        # QA agents' generated tokens of this batch (each result holds every row of the batch)
        eff.add(time.perf_counter() - t0, len(idx), sum(len(t) for g in outs[0].results.values() for t in g.tokens))
    means = results.means()
    for line in format_final_report(means):
        logger.info(line)
    means.update(eff.summary())
    for line in format_efficiency_report(means):
        logger.info(line)
    for name, d in agent_tps.items():
        if d["gen"]:
            g, a = sum(d["gen"]) / len(d["gen"]), sum(d["all"]) / len(d["all"])
            means[f"tps_gen_{name}"], means[f"tps_all_{name}"] = g, a
            logger.info(f"TPS {name:<14}→ {g:.2f} generated / {a:.2f} prompt+generated tok/s")
    return means


def main(argv: Optional[List[str]] = None) -> dict:
    p = add_runtime_args(add_reference_args(argparse.ArgumentParser(description=__doc__), "combiner"))
    args = p.parse_args(argv)
    rt = pop_runtime(args)
    if args.config is not None and not os.path.exists(args.config):
        logger.error(f"Config file not found: {args.config}")      # combine_model_fp_updated.py:158-160
        sys.exit(1)
    cfg = apply_overrides(load_config(args.config), args)
    if cfg.agents:
        qa = [(a.name, a.model, a.precision, a.quant, a.gpus) for a in cfg.agents]
    else:  # the reference's three fixed roles (combine_model_fp_updated.py:174-176)
        qa = [("phi_model", cfg.phi_model or "microsoft/phi-2", "fp16"),
              ("pythia_model", cfg.pythia_model or "EleutherAI/pythia-1b", "fp16")]
    refiner = ("refiner_model", cfg.refiner_model or "meta-llama/Llama-3.2-1B-Instruct", "bf16")
    return run_ensemble(cfg, rt, qa, refiner)


if __name__ == "__main__":
    main()

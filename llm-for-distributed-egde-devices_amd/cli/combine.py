"""Multi-agent ensemble evaluator — the reference's combiner scripts on edgellm.

    python -m edgellm.cli.combine --config config.yaml [--max_new_tokens 200 ...]            # C4/C7 (fp)
    python -m edgellm.cli.combine --config config.yaml --quant llm_int8                      # C5/C6 (bnb-style INT8)
    python -m edgellm.cli.combine --config config.yaml --quant w8a8_smoothquant --merge vote  # north star

Same YAML keys / 13 CLI flags / log lines as Code/Base Models/combine_model_fp_updated.py:138-232
(and Code/Quantised Models/combiner_quant_updated.py).  Agents run concurrently on separate
GPUs; the refiner merges (or a majority vote).  Per-sample metrics: ROUGE-1/2/L, BERTScore,
BLEU, cosine, confidence (scored with the refiner), combo TPS = mean of the QA agents' TPS.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import List, Optional

import torch

from ..config import add_reference_args, apply_overrides, load_config, RunConfig
from ..data import load_qa
from ..engine import Generator, SamplingParams
from ..eval import Embedder, MetricSuite, ProgressLog, Results
from ..models.registry import load_model
from ..orchestrator import Agent, Orchestrator, RefineMerge, VoteMerge
from ..utils.log import format_final_report, get_logger
from .common import add_runtime_args, pick_devices, pop_runtime

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
               cpu_prompt: bool = False) -> Agent:
    model, tok, source = load_model(model_id, precision, quant, device, rt.get("base_model_path"))
    logger.info(f"{name}: {source} on {device} ({quant})")
    gen = Generator(model, max_batch=1, max_seq=rt.get("max_seq", 2048))
    return Agent(name, gen, tok, sampling, cpu_prompt)


def run_ensemble(cfg: RunConfig, rt: dict, qa_specs, refiner_spec, cpu_variant: bool = False) -> dict:
    quant = rt.get("quant") or cfg.quant.mode
    devices = pick_devices(rt.get("devices"))
    s = cfg.sampling
    sampling = SamplingParams(s.max_new_tokens, s.temperature, s.top_k, s.top_p, s.repetition_penalty, s.do_sample)
    logger.info("Loading dataset...")
    rows = load_qa(cfg.dataset_name, cfg.dataset_split, cfg.dataset_path, rt.get("num_samples"))
    logger.info("Loading models...")
    agents = [make_agent(n, mid, prec, quant, devices[i % len(devices)], sampling, rt, cpu_variant)
              for i, (n, mid, prec) in enumerate(qa_specs)]
    merge_kind = rt.get("merge") or cfg.merge
    refiner = None
    if merge_kind == "refine" or refiner_spec is not None:
        rn, rid, rprec = refiner_spec
        refiner = make_agent(rn, rid, rprec, quant, devices[len(agents) % len(devices)], sampling, rt)
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
    progress = ProgressLog(rt.get("progress"))
    done = progress.done()
    results = Results()
    logger.info("Starting evaluation loop...")
    for i, sample in enumerate(rows):
        if i in done:
            results.add({k: done[i][k] for k in done[i] if k not in ("index",)})
            continue
        q, ref = sample["query"], sample["answer"]
        logger.info(f"Processing question: {q}")
        res = orch.answer(q, ref, seed=rt.get("seed", 0) + i)
        for name, ans in res.answers.items():
            logger.info(f"Answer from {name}: {ans[:100]}...")
            if cpu_variant:
                logger.info(f"[Q{i + 1}] {name} TPS: {res.tps[name]:.2f} tokens/sec")
        logger.info(f"Refined response: {res.final[:100]}...")
        m = suite.score(res.final, ref, scorer.generator.model, scorer.tokenizer, tps=res.combo_tps)
        if m["rouge1"] == 0.0 and m["tps"] == 0.0:
            logger.error("Error in evaluation: metrics zeroed for this sample")
        results.add(m)
        progress.append(i, m)
        if rt.get("metrics_jsonl"):
            with open(rt["metrics_jsonl"], "a") as f:
                f.write(json.dumps({"index": i, **m, "agent_tps": res.tps, "wall_s": res.wall_s}) + "\n")
        if cpu_variant:
            logger.info(f"[Q{i + 1}] Total time: {res.wall_s:.2f} sec\n")
    means = results.means()
    for line in format_final_report(means):
        logger.info(line)
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
        qa = [(a.name, a.model, a.precision) for a in cfg.agents]
    else:  # the reference's three fixed roles (combine_model_fp_updated.py:174-176)
        qa = [("phi_model", cfg.phi_model or "microsoft/phi-2", "fp16"),
              ("pythia_model", cfg.pythia_model or "EleutherAI/pythia-1b", "fp16")]
    refiner = ("refiner_model", cfg.refiner_model or "meta-llama/Llama-3.2-1B-Instruct", "bf16")
    return run_ensemble(cfg, rt, qa, refiner)


if __name__ == "__main__":
    main()

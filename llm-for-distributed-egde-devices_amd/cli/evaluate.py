"""Single-model evaluator — the reference's ``Llama_bf16_updated.py`` / ``phi2-pythia_fp_updated.py``
/ ``models_quant_updated.py`` on edgellm.

    python -m edgellm.cli.evaluate --config config.yaml --models meta-llama/Llama-3.2-1B-Instruct
    python -m edgellm.cli.evaluate --config config.yaml --models microsoft/phi-2 --quant llm_int8

Flags: --config --models --dataset_name --dataset_split --max_new_tokens --temperature --top_k
--top_p --repetition_penalty (Llama_bf16_updated.py:138-146).  Per model: generate for every
sample, score the 7 quality metrics (confidence with the model itself, Llama_bf16_updated.py:111)
and TPS counting prompt + generated tokens (:89-90), then log the 9 means.
"""
from __future__ import annotations

import argparse
import os
import time
from typing import List, Optional

from ..config import add_reference_args, apply_overrides, load_config
from ..data import load_qa
from ..engine import SamplingParams
from ..eval import EfficiencyMeter, MetricSuite, Results
from ..models.registry import load_model
from ..orchestrator.prompts import qa_prompt
from ..parallel.split import agent_devices, split_model
from ..utils.log import format_efficiency_report, format_single_model_report, get_logger
from .combine import build_embedder
from .common import (add_runtime_args, build_generator, build_pp_engine, pick_devices, pop_runtime, pp_launch,
                     resolve_runtime)

logger = get_logger("evaluate")


def evaluate_model(model_id: str, rows, cfg, rt) -> dict:
    """The reference's per-model loop (Llama_bf16_updated.py:96-134).  ``pp_size`` > 1 splits the
    model's layers over that many GPUs (its ``device_map="auto"``, :31); ``batch_size`` > 1
    decodes that many questions together (TPS per sample = its tokens incl. prompt / the batch's
    wall time)."""
    logger.info(f"\n--- Evaluating Model: {model_id} ---")
    rt = resolve_runtime(cfg, rt)
    quant = rt.get("quant") or cfg.quant.mode
    precision = rt.get("precision") or "bf16"
    bs = max(1, int(rt.get("batch_size") or 1))
    launch = pp_launch(rt)
    if launch is not None:
        # torchrun: one pipeline stage per rank; rank 0 drives the loop, the others serve it
        from ..parallel.pp_engine import serve_workers, stop_workers
        gen, tok, source, bounds = build_pp_engine(model_id, precision, quant, rt, launch, tag=0, max_batch=bs)
        if launch[0] != 0:
            serve_workers({0: gen})
            return {}
        logger.info(f"{model_id}: {source} pipelined over {launch[1]} ranks at layers {bounds} ({quant})")
        dev = launch[2]
        devs = [dev]
        model = gen.model                    # confidence scored through the pipeline
        out = _evaluate_loop(model_id, rows, cfg, rt, gen, model, tok, dev, devs, bs)
        stop_workers(gen)                    # (not on an exception: torchrun tears the workers down)
        return out
    dev = pick_devices(rt.get("devices"))[0]
    devs = agent_devices(None, dev, int(rt.get("pp_size") or 1))
    model, tok, source = load_model(model_id, precision, quant, devs[0], rt.get("base_model_path"))
    if len(devs) > 1:
        model = split_model(model, devs)
        logger.info(f"{model_id}: {source} split over {[str(d) for d in devs]} at layers {model.bounds} ({quant})")
    else:
        logger.info(f"{model_id}: {source} ({quant})")
    gen = build_generator(model, rt, max_batch=bs)
    return _evaluate_loop(model_id, rows, cfg, rt, gen, model, tok, dev, devs, bs)


def _evaluate_loop(model_id, rows, cfg, rt, gen, model, tok, dev, devs, bs) -> dict:
    s = cfg.sampling
    sp = SamplingParams(s.max_new_tokens, s.temperature, s.top_k, s.top_p, s.repetition_penalty, s.do_sample)
    suite = MetricSuite(build_embedder(cfg.embedder_model, rt.get("base_model_path"), dev))
    res_all = Results()
    eff = EfficiencyMeter(devs)
    eos = getattr(tok, "eos_token_id", None)
    for j0 in range(0, len(rows), bs):
        batch = rows[j0:j0 + bs]
        t0 = time.perf_counter()
        ids = [tok.encode(qa_prompt(smp["query"]))[-(gen.max_seq - sp.max_new_tokens):] for smp in batch]
        r = gen.generate(ids, sp, seed=rt.get("seed", 0) + j0, eos_token_id=eos)
        for i, (smp, pid, out) in enumerate(zip(batch, ids, r.tokens)):
            text = tok.decode((pid + out) if not rt.get("no_legacy_decode") else out, skip_special_tokens=True).strip()
            # prompt + generated tokens / generate wall time (Llama_bf16_updated.py:89-90)
            tps = (len(pid) + len(out)) / r.elapsed_s if r.elapsed_s > 0 else 0.0
            res_all.add(suite.score(text, smp["answer"], model, tok, tps=tps))
        eff.add(time.perf_counter() - t0, len(batch), r.num_generated)
    means = res_all.means()
    for line in format_single_model_report(means):
        logger.info(line)
    means.update(eff.summary())
    for line in format_efficiency_report(means):
        logger.info(line)
    return means


def main(argv: Optional[List[str]] = None):
    p = add_runtime_args(add_reference_args(argparse.ArgumentParser(description=__doc__), "single"))
    args = p.parse_args(argv)
    rt = pop_runtime(args)
    cfg = apply_overrides(load_config(args.config if args.config and os.path.exists(args.config) else None), args)
    models = cfg.models or ["meta-llama/Llama-3.2-1B-Instruct"]
    rows = load_qa(cfg.dataset_name, cfg.dataset_split, cfg.dataset_path, rt.get("num_samples"))
    return {m: evaluate_model(m, rows, cfg, rt) for m in models}


if __name__ == "__main__":
    main()

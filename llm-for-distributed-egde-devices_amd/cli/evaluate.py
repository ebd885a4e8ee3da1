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
from typing import List, Optional

from ..config import add_reference_args, apply_overrides, load_config
from ..data import load_qa
from ..engine import Generator, SamplingParams
from ..eval import MetricSuite, Results
from ..models.registry import load_model
from ..orchestrator.prompts import qa_prompt
from ..utils.log import format_single_model_report, get_logger
from .combine import build_embedder
from .common import add_runtime_args, pick_devices, pop_runtime

logger = get_logger("evaluate")


def evaluate_model(model_id: str, rows, cfg, rt) -> dict:
    logger.info(f"\n--- Evaluating Model: {model_id} ---")
    dev = pick_devices(rt.get("devices"))[0]
    quant = rt.get("quant") or cfg.quant.mode
    precision = rt.get("precision") or "bf16"
    model, tok, source = load_model(model_id, precision, quant, dev, rt.get("base_model_path"))
    logger.info(f"{model_id}: {source} ({quant})")
    gen = Generator(model, max_batch=1, max_seq=rt.get("max_seq", 2048))
    s = cfg.sampling
    sp = SamplingParams(s.max_new_tokens, s.temperature, s.top_k, s.top_p, s.repetition_penalty, s.do_sample)
    suite = MetricSuite(build_embedder(cfg.embedder_model, rt.get("base_model_path"), dev))
    res_all = Results()
    for i, sample in enumerate(rows):
        ids = tok.encode(qa_prompt(sample["query"]))
        ids = ids[-(gen.max_seq - sp.max_new_tokens):]
        r = gen.generate([ids], sp, seed=rt.get("seed", 0) + i, eos_token_id=getattr(tok, "eos_token_id", None))
        text = tok.decode((ids + r.tokens[0]) if not rt.get("no_legacy_decode") else r.tokens[0],
                          skip_special_tokens=True).strip()
        res_all.add(suite.score(text, sample["answer"], model, tok, tps=r.tps_incl_prompt()))
    means = res_all.means()
    for line in format_single_model_report(means):
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

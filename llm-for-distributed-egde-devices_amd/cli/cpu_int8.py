"""CPU INT8 edge ensemble — the reference's ``Code/C-DAC Server/try.py`` on edgellm.

All three models on CPU with torch dynamic qint8 linears (try.py:198-206), the CPU prompt
variant (try.py:239-243), fixed sampling max_new_tokens=180, T=0.5, top-k 30, top-p 0.85,
repetition 1.2 (try.py:308-314), per-agent TPS logged per question, combo TPS averaging all three
agents including the refiner (try.py:323), total question time logged (:337).
"""
from __future__ import annotations

import argparse
from typing import List, Optional

from ..config import RunConfig
from .combine import run_ensemble
from .common import add_runtime_args, pop_runtime


def main(argv: Optional[List[str]] = None):
    p = add_runtime_args(argparse.ArgumentParser(description=__doc__))
    p.add_argument("--dataset_path", default=None, help="natural_questions_1000.csv")
    p.add_argument("--phi_model", default="microsoft/phi-2")
    p.add_argument("--pythia_model", default="EleutherAI/pythia-1b")
    p.add_argument("--refiner_model", default="meta-llama/Llama-3.2-1B-Instruct")
    p.add_argument("--embedder_model", default="sentence-transformers/all-MiniLM-L6-v2")
    args = p.parse_args(argv)
    rt = pop_runtime(args)
    rt.setdefault("quant", None)
    rt["quant"] = rt["quant"] or "cpu_dynamic"
    rt["devices"] = rt.get("devices") or "cpu"
    cfg = RunConfig()
    cfg.dataset_path = args.dataset_path
    cfg.dataset_name = args.dataset_path or cfg.dataset_name
    cfg.embedder_model = args.embedder_model
    s = cfg.sampling
    s.max_new_tokens, s.temperature, s.top_k, s.top_p, s.repetition_penalty = 180, 0.5, 30, 0.85, 1.2
    qa = [("Phi-2", args.phi_model, "fp32"), ("Pythia", args.pythia_model, "fp32")]
    return run_ensemble(cfg, rt, qa, ("Refiner", args.refiner_model, "fp32"), cpu_variant=True)


if __name__ == "__main__":
    main()

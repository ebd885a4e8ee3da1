"""Shared CLI plumbing: device selection, argument groups beyond the reference's flags."""
from __future__ import annotations

import argparse
from typing import List

import torch


def add_runtime_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    g = p.add_argument_group("edgellm runtime (not in the reference)")
    g.add_argument("--quant", default=None, choices=["none", "w8a8_smoothquant", "w8a8", "llm_int8", "cpu_dynamic"],
                   help="quantisation mode (default: none, or from YAML quant.mode)")
    g.add_argument("--precision", default=None, help="fp16|bf16|fp32 (GPU runs bf16)")
    g.add_argument("--devices", default=None, help="comma list, e.g. cuda:0,cuda:1 (agents round-robin)")
    g.add_argument("--num_samples", type=int, default=None, help="evaluate only the first N samples")
    g.add_argument("--seed", type=int, default=0, help="sampling seed (the reference sets none)")
    g.add_argument("--max_seq", type=int, default=2048, help="KV-cache capacity per sequence")
    g.add_argument("--progress", default=None, help="JSONL progress file (resume after a crash)")
    g.add_argument("--base_model_path", default=None, help="directory holding downloaded checkpoints")
    g.add_argument("--no_legacy_decode", action="store_true",
                   help="score only generated text (the reference decodes prompt + answer)")
    g.add_argument("--no_reference_in_refiner", action="store_true",
                   help="do not leak the gold answer into the refiner prompt")
    g.add_argument("--merge", default=None, choices=["refine", "vote"], help="ensemble merge (default refine)")
    g.add_argument("--serial", action="store_true", help="run agents one after another (reference behaviour)")
    g.add_argument("--headinfer_heads", type=int, default=None, help="KV heads resident on GPU (HeadInfer)")
    g.add_argument("--metrics_jsonl", default=None, help="append structured per-sample metrics here")
    return p


def pick_devices(spec: str = None) -> List[torch.device]:
    if spec:
        return [torch.device(s.strip()) for s in spec.split(",") if s.strip()]
    if torch.cuda.is_available():
        return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    return [torch.device("cpu")]


def pop_runtime(args: argparse.Namespace) -> dict:
    """Remove runtime-only keys so the remaining namespace is the reference's flag set."""
    keys = ["quant", "precision", "devices", "num_samples", "seed", "max_seq", "progress", "base_model_path",
            "no_legacy_decode", "no_reference_in_refiner", "merge", "serial", "headinfer_heads", "metrics_jsonl"]
    return {k: args.__dict__.pop(k) for k in keys if k in args.__dict__}

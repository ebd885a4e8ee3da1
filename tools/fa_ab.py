#!/usr/bin/env python
"""Interleaved A/B of flash-prefill launch variants at the TTFT-relevant causal shapes: several rounds
in one process, variants rotated each round, median TF/s per variant.

  --knob stagger: wave schedules (tune ``prefill_fa`` second value as the binding reads it: 2 staggered,
    the default, 1 lockstep).  Round 4 (profiles/fa_schedule_ab_r4.json): staggered 3.5-5.5 % over
    lockstep at D = 128, lockstep +1 % at D = 64.
  --knob sm: static s_setprio 1 for waves 4-7 and the deferred-max threshold (tune ``prefill_fa_sm``).
  (Round 5 also measured hoisted loop-invariant DMA / LDS offsets, a buffer-resource DMA and the
  permlane32 half reductions: profiles/fa_v2_forms_ab_r5.json; only the permlane form was kept.)
  (The scalar-base DMA addressing was A/B'd the same way: profiles/fa_saddr_ab_r5.json.)
  --knob order: workgroup order (tune ``prefill_fa_order``: 1 longest query tiles first over all heads,
    the default, 0 longest first per head).  The shapes include the 4K chunks of a 32K prompt.

    python tools/fa_ab.py [--knob order] [--rounds 5] [--out file.json]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_ops import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--knob", default="stagger", choices=["stagger", "order", "sm"])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = ops.ext()
    rows = []
    shapes = [(32768, 32, 8, 0, 128), (4096, 32, 8, 28672, 128), (8192, 32, 8, 0, 128),
              (2048, 32, 32, 0, 128), (1024, 32, 8, 0, 64)]
    if a.knob == "order":
        shapes = [(4096, 32, 8, 0, 128), (4096, 32, 8, 12288, 128)] + shapes
    names = {"stagger": {2: "staggered", 1: "lockstep"}, "order": {1: "all_heads", 0: "per_head"},
             "sm": {(0, 0): "exact", (1, 0): "prio", (0, 8): "thr8", (1, 8): "prio_thr8"}}[a.knob]
    order = list(names)

    def setk(v):
        if a.knob == "stagger":
            C.tune("prefill_fa", 2, v)
        elif a.knob == "order":
            C.tune("prefill_fa", 2, 0)
            C.tune("prefill_fa_order", v, 0)
        else:
            C.tune("prefill_fa", 2, 0)
            C.tune("prefill_fa_sm", *v)
    for T, Hq, Hkv, s0, D in shapes:
        q = torch.randn(1, T, Hq, D, device=dev).bfloat16()
        kc = torch.randn(1, Hkv, s0 + T, D, device=dev).bfloat16()
        vc = torch.randn_like(kc)
        sp = torch.full((1,), s0, dtype=torch.int32, device=dev)
        flops = 4 * T * (s0 + T / 2) * D * Hq
        res = {k: [] for k in order}
        for r in range(a.rounds):
            k = r % len(order)
            for stg in order[k:] + order[:k]:
                setk(stg)
                t = timeit(lambda: C.prefill_attn(q, kc, vc, sp, 1 / math.sqrt(D), True), iters=5,
                           per_graph=2 if T >= 16384 else 10)
                res[stg].append(flops / t / 1e6)
        C.tune("prefill_fa", 1, 0)
        C.tune("prefill_fa_order", 1, 0)
        C.tune("prefill_fa_sm", 0, 0)
        row = dict(T=T, start=s0, Hq=Hq, Hkv=Hkv, D=D, knob=a.knob)
        for stg, name in names.items():
            v = sorted(res[stg])
            row[name + "_TFLOPs_median"] = round(v[len(v) // 2], 1)
            row[name + "_TFLOPs_all"] = [round(x, 1) for x in res[stg]]
        rows.append(row)
        print(json.dumps(row), flush=True)
        del q, kc, vc
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""A/B of the 256-row decode GEMM forms at Llama-2-7B shapes, interleaved in one process: ring2
(weights through the LDS-DMA ring, tune r256_wreg 0) against the weights-in-VGPR kernel
(gemm_i8_wreg.hip, r256_wreg 4 / 6 = stages in flight).  Weights rotate over enough copies that
every call streams them from HBM.

    python tools/wreg_ab.py [--rounds 5] [--out gpurun_out/wreg_ab.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402
from bench_ops import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = ops.ext()
    shapes = {"qkv": (12288, 4096, "out", (0, 4, 6)), "gate_up": (22016, 4096, "gluq", (0, 4)),
              "lm_head_like": (32000, 4096, "out", (0, 4, 6))}
    rows = []
    for name, (N, K, kind, forms) in shapes.items():
        ncopy = max(2, (1 << 30) // (N * K) + 1)
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
        sw = torch.rand(N, device=dev) * 0.01
        qx = torch.randint(-127, 128, (a.M, K), dtype=torch.int8, device=dev)
        sx = torch.rand(a.M, device=dev) * 0.01
        ctr = [0]

        def call():
            ctr[0] = (ctr[0] + 1) % ncopy
            if kind == "gluq":
                return C.w8a8_gemm_gluq(qx, sx, wps[ctr[0]], sw, None, N, K)
            return C.w8a8_gemm(qx, sx, wps[ctr[0]], sw, None, N, K)

        res = {f: [] for f in forms}
        for _ in range(a.rounds):
            for f in forms:
                C.tune("r256_wreg", f, 0)
                res[f].append(timeit(call, iters=10, per_graph=ncopy))
        C.tune("r256_wreg", 0, 0)
        row = dict(op="w8a8_rows256_wreg_ab", shape=name, M=a.M, N=N, K=K, weight_MB=round(N * K / 1e6, 1))
        for f, ts in res.items():
            key = "ring2" if f == 0 else f"wreg{f}"
            row[f"{key}_us"] = round(sorted(ts)[len(ts) // 2], 2)
            row[f"{key}_min_us"] = round(min(ts), 2)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del wps
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()

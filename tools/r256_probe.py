#!/usr/bin/env python
"""Minimal driver for counter passes on the 256-row decode GEMMs (Llama-2-7B W8A8 shapes):
runs qkv, o (grouped scales, split-K), gate_up (SwiGLU + quant) and down (grouped scales,
split-K) ``--iters`` times each on rotated, cache-cold weight copies, nothing else on the GPU.

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES ... -d gpurun_out/pmc -- python3 tools/r256_probe.py
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402

SHAPES = {"qkv": (12288, 4096, "out"), "o": (4096, 4096, "part"), "gate_up": (22016, 4096, "gluq"),
          "down": (4096, 11008, "part")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--only", default=None)
    ap.add_argument("--tune", action="append", default=[], help="name=a[,b] (ext().tune)")
    a = ap.parse_args()
    C = ops.ext()
    for t in a.tune:
        name, vals = t.split("=")
        v = [int(x) for x in vals.split(",")] + [0]
        C.tune(name, v[0], v[1])
    dev = torch.device("cuda:0")
    M = a.rows
    for name, (N, K, kind) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        ncopy = max(2, (1 << 30) // (N * K) + 1)
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
        sw = torch.rand(N, device=dev) * 0.01
        qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        sx = (torch.rand(K // 64, (M + 15) // 16 * 16, device=dev) if kind == "part" else torch.rand(M, device=dev)) * 0.01
        for i in range(a.iters):
            wp = wps[i % ncopy]
            if kind == "gluq":
                C.w8a8_gemm_gluq(qx, sx, wp, sw, None, N, K)
            elif kind == "part":
                C.w8a8_gemm_splitk(qx, sx, wp, sw, None, N, K, 0)
            else:
                C.w8a8_gemm(qx, sx, wp, sw, None, N, K)
        torch.cuda.synchronize()
        del wps
        print(name, "done", flush=True)


if __name__ == "__main__":
    main()

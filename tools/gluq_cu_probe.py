#!/usr/bin/env python
"""Batch-1 quantising gate_up GEMV: time per weight MB against the workgroup count (one workgroup
per 64 output features = 8 tiles).  Llama-2-7B's 11008 features give 172 workgroups on 256 CUs;
the probe sweeps F so the grid spans 128..320 workgroups at K = 4096 (cache-cold weight copies).

    python tools/gluq_cu_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_ops import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    C = ops.ext()
    K = 4096
    qx = torch.randint(-127, 128, (1, K), dtype=torch.int8, device=dev)
    sx = torch.rand(1, device=dev) * 0.01
    for wgs in (128, 160, 172, 192, 224, 256, 288, 320):
        F = wgs * 64
        N = 2 * F
        ncopy = max(2, (1 << 30) // (N * K) + 1)
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
        sw = torch.rand(N, device=dev) * 0.01
        ctr = [0]

        def call():
            ctr[0] = (ctr[0] + 1) % ncopy
            return C.w8a8_gemm_gluq(qx, sx, wps[ctr[0]], sw, None, N, K)
        us = min(timeit(call, iters=10, per_graph=ncopy) for _ in range(3))
        print(json.dumps(dict(workgroups=wgs, N=N, K=K, us=round(us, 2), TBps=round(N * K / us / 1e6, 2))), flush=True)
        del wps, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

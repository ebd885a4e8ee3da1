#!/usr/bin/env python
"""One prefill INT8 GEMM form at one shape, repeated: a short, fixed workload for rocprofv3 PMC
passes (kernel-trace / counters), plus the same shape through torch._int_mm (hipBLASLt int8) as
the library reference point.

    python tools/pgemm_probe.py --x32 2 --M 16384 --N 12288 --K 4096 --iters 20

--x32: 0 the 128 x 256 16x16x64 ring kernel, 2 the 256 x 256 32x32x32 kernel, 1 the launcher's
choice (x32 from 512 tiles).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--x32", type=int, default=1)
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=12288)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--intmm", action="store_true", help="also time torch._int_mm (hipBLASLt)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = ops.ext()
    M, N, K = a.M, a.N, a.K
    x = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
    wp = ops.pack_int8_weight(w)
    sx, sw = torch.rand(M, device=dev) * 0.01, torch.rand(N, device=dev) * 0.01
    C.tune("prefill_x32", a.x32, 0)
    fns = {"edge": lambda: C.w8a8_gemm(x, sx, wp, sw, None, N, K)}
    if a.intmm:
        wt = w.t()                           # [K, N] column-major view of the [N, K] weight
        fns["int_mm"] = lambda: torch._int_mm(x, wt)
    for name, fn in fns.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(f"{name} x32={a.x32} M={M} N={N} K={K}: {us:.1f} us  {2 * M * N * K / us / 1e6:.0f} TOPS", flush=True)


if __name__ == "__main__":
    main()

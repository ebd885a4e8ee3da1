#!/usr/bin/env python
"""A few flash-prefill calls at one shape, for counter passes (rocprofv3 --pmc) on fa_kernel.

    python tools/fa_probe.py --T 32768 --start 0 --calls 3 [--tune prefill_fa_sm=0,8]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=32768)
    ap.add_argument("--start", type=int, default=0)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--tune", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = ops.ext()
    ops.apply_tune(a.tune)
    C.tune("prefill_fa", 2, 0)
    q = torch.randn(1, a.T, a.Hq, a.D, device=dev).bfloat16()
    kc = torch.randn(1, a.Hkv, a.start + a.T, a.D, device=dev).bfloat16()
    vc = torch.randn_like(kc)
    sp = torch.full((1,), a.start, dtype=torch.int32, device=dev)
    for _ in range(a.calls):
        C.prefill_attn(q, kc, vc, sp, 1 / math.sqrt(a.D), True)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()

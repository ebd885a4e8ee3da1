#!/usr/bin/env python
"""CU-partition lab: does splitting the chip's CUs between decode attention (HBM-bound) and the
256-row decode GEMMs (bound per CU) let one lane's attention run beside the other lane's GEMMs?

Two 256-row lanes today overlap ~14 % (docs/BENCHMARKS.md): both lanes' kernels want every CU.
Here attention and GEMMs go to streams created with hipExtStreamCreateWithCUMask (CU sets of c and
256 - c CUs) and are timed alone and concurrently, against the unmasked pair.

Kernels (Llama-2-7B, 256 rows): fused decode attention over a bf16 KV cache of `ctx` tokens (32
heads x 128), and a W8A8 GEMM sequence of one layer (qkv, o split-K, gate_up + SwiGLU + int8, down
split-K) on the production launchers.  Each side repeats `reps` layers inside one timed region.

    python tools/cu_split_lab.py --ctx 150 --reps 8 --splits 64,96,128
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from edgellm import ops  # noqa: E402
from edgellm.ops import _ref  # noqa: E402

_hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(cus, n_total: int = 256) -> torch.cuda.ExternalStream:
    """A HIP stream restricted to the CU indices ``cus`` (hipExtStreamCreateWithCUMask)."""
    words = (ctypes.c_uint32 * ((n_total + 31) // 32))()
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = _hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), words)
    assert rc == 0, f"hipExtStreamCreateWithCUMask failed: {rc}"
    return torch.cuda.ExternalStream(s.value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=150)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--splits", default="64,96,128")
    ap.add_argument("--layout", default="block", choices=["block", "stride"],
                    help="block: CUs [0, c) vs [c, 256); stride: every k-th CU to attention")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = ops.ext()
    props = torch.cuda.get_device_properties(dev)
    NCU = props.multi_processor_count
    B, Hq, D, H, F = 256, 32, 128, 4096, 11008
    S = a.ctx + 8
    g = torch.Generator(device=dev).manual_seed(0)
    kc = torch.randn(B, Hq, S, D, device=dev, generator=g).bfloat16()
    vc = torch.randn(B, Hq, S, D, device=dev, generator=g).bfloat16()
    qkv = torch.randn(B, 3 * H, device=dev, generator=g).bfloat16()
    lens = torch.full((B,), a.ctx, dtype=torch.int32, device=dev)
    pos = lens - 1
    rope = _ref.rope_tables(D, 4096, 10000.0, device=dev)

    def attn():
        for _ in range(a.reps):
            C.decode_attn_fused(qkv, pos, rope, kc, vc, lens, Hq, 1 / math.sqrt(D), S, D, True)

    def w(n, k):
        wi = torch.randint(-127, 128, (n, k), dtype=torch.int8, device=dev, generator=g)
        return ops.pack_int8_weight(wi), torch.rand(n, device=dev, generator=g) * 0.01 + 1e-3
    wq, wo, wgu, wd = w(3 * H, H), w(H, H), w(2 * F, H), w(H, F)
    xa = torch.randint(-127, 128, (B, H), dtype=torch.int8, device=dev, generator=g)
    xs = torch.rand(B, device=dev, generator=g) * 0.01
    xg = torch.rand(H // 64, B, device=dev, generator=g) * 0.01           # grouped scales [K/64, Mpad]
    xf = torch.randint(-127, 128, (B, F), dtype=torch.int8, device=dev, generator=g)
    xfg = torch.rand(F // 64, B, device=dev, generator=g) * 0.01

    def gemms():
        for _ in range(a.reps):
            C.w8a8_gemm(xa, xs, wq[0], wq[1], None, 3 * H, H)
            C.w8a8_gemm_splitk(xa, xg, wo[0], wo[1], None, H, H, 0)
            C.w8a8_gemm_gluq(xa, xs, wgu[0], wgu[1], None, 2 * F, H)
            C.w8a8_gemm_splitk(xf, xfg, wd[0], wd[1], None, H, F, 0)

    def timed(pairs, iters=5):
        """pairs: [(fn, stream)] run concurrently; returns ms of the slowest (events on each)."""
        for fn, st in pairs:                                     # warm
            with torch.cuda.stream(st):
                fn()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(iters):
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record()
            ends = []
            for fn, st in pairs:
                st.wait_event(t0)
                with torch.cuda.stream(st):
                    fn()
                    e = torch.cuda.Event(enable_timing=True)
                    e.record()
                    ends.append(e)
            torch.cuda.synchronize()
            best = min(best, max(t0.elapsed_time(e) for e in ends))
        return round(best, 3)

    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    base = dict(ncu=NCU, ctx=a.ctx, reps=a.reps)
    print(json.dumps(dict(base, case="attn_alone", ms=timed([(attn, s1)]))), flush=True)
    print(json.dumps(dict(base, case="gemm_alone", ms=timed([(gemms, s1)]))), flush=True)
    print(json.dumps(dict(base, case="both_unmasked", ms=timed([(attn, s1), (gemms, s2)]))), flush=True)
    for c in [int(x) for x in a.splits.split(",")]:
        if a.layout == "block":
            ca = list(range(c))
        else:
            k = max(1, round(NCU / c))
            ca = list(range(0, NCU, k))[:c]
        cg = [i for i in range(NCU) if i not in set(ca)]
        sa, sg = masked_stream(ca, NCU), masked_stream(cg, NCU)
        row = dict(base, case="split", attn_cus=len(ca), gemm_cus=len(cg), layout=a.layout,
                   attn_ms=timed([(attn, sa)]), gemm_ms=timed([(gemms, sg)]),
                   both_ms=timed([(attn, sa), (gemms, sg)]))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

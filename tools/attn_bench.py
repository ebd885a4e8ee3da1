#!/usr/bin/env python
"""Decode-attention microbenchmark: bf16 vs int8 KV cache, the model's fused launch (RoPE +
append + attention + int8 output) at decode shapes; several cache copies rotate so every call
streams its K/V from HBM (the per-layer caches of a real step never share lines).

    python tools/attn_bench.py [--out profiles/attn_bench.json] [--shapes 128x160,...]
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
from edgellm.ops import _ref  # noqa: E402


def timeit(fns, iters=20):
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for f in fns:
            f()
    g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    ev[0].record()
    for i in range(iters):
        g.replay()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(iters))
    return ts[len(ts) // 2] * 1e3 / len(fns)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="128x160,128x512,64x160,16x2048,1x160,1x4096")
    ap.add_argument("--heads", default="32x32")        # Hq x Hkv
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--copies", type=int, default=0, help="cache copies rotated (0: enough for > 512 MB)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="bf16,int8,int8wave",
                    help="bf16 | bf16u8 (8 key groups per wave per chunk) | int8 (workgroup-per-head split form) | "
                         "int8wave (wave-per-head form); a kind may repeat (interleaved A/B)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    Hq, Hkv = (int(x) for x in a.heads.split("x"))
    D = a.D
    rows = []
    for shp in a.shapes.split(","):
        B, L = (int(x) for x in shp.split("x"))
        S = L + 8
        per16 = 2 * B * Hkv * S * D * 2
        n = a.copies or max(2, min(16, int(math.ceil(600e6 / per16))))
        qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).bfloat16()
        sl = torch.full((B,), L, dtype=torch.int32, device=dev)
        pos = sl - 1
        rope = ops.rope_tables(D, S, 10000.0, device=dev)
        for kind in a.only.split(","):
            ops.ext().tune("attn8_wave_max", 1024 if kind == "int8wave" else 0, 0)
            # bf16u8: the barrier-free MHA form with 8 key groups per wave per chunk (tune decode_attn_unroll)
            ops.ext().tune("decode_attn_unroll", 8 if kind == "bf16u8" else 4, 0)
            caches = []
            for _ in range(n):
                k = torch.randn(B, Hkv, S, D, device=dev).bfloat16()
                v = torch.randn_like(k)
                if kind.startswith("int8"):
                    kq, ks = _ref.quant_kv_rows(k)
                    vq, vs = _ref.quant_kv_rows(v)
                    caches.append((kq, vq, ks.contiguous(), vs.contiguous()))
                else:
                    caches.append((k, v))
            if kind.startswith("int8"):
                fns = [lambda c=c: ops.decode_attention_fused_i8(qkv, pos, rope, c[0], c[1], c[2], c[3], sl, Hq,
                                                                 1 / math.sqrt(D), L, D, True) for c in caches]
                nbytes = 2 * B * Hkv * L * (D + 4)
            else:
                fns = [lambda c=c: ops.decode_attention_fused(qkv, pos, rope, c[0], c[1], sl, Hq, 1 / math.sqrt(D),
                                                              L, D, True) for c in caches]
                nbytes = 2 * B * Hkv * L * D * 2
            us = timeit(fns)
            rows.append(dict(op=f"decode_attn_fused_{kind}", B=B, ctx=L, Hq=Hq, Hkv=Hkv, D=D, copies=n,
                             us=round(us, 2), TBps=round(nbytes / us / 1e6, 2)))
            print(json.dumps(rows[-1]), flush=True)
            del caches, fns
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Per-op microbenchmarks of the HIP kernels at Llama-2-7B decode shapes (MI355X).

Reports time and achieved HBM bandwidth per op; tuning sweeps of the INT8 GEMV (waves per
workgroup x unroll) are timed interleaved in one process (cdna guide §5.4 rule 24) on random
data.  Writes a JSON summary (``--out``).

    python tools/bench_ops.py --out profiles/bench_ops.json
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402


GLOBAL_TUNE = []   # --tune settings; re-applied whenever a sweep resets a knob to automatic


def tune(C, name, a, b=0):
    """Set a tuning knob; (0, 0) means automatic unless --tune pinned that knob."""
    for n, va, vb in GLOBAL_TUNE:
        if n == name and a == 0 and b == 0:
            a, b = va, vb
    C.tune(name, a, b)


def timeit(fn, iters=50, warm=3, per_graph=20):
    """Median per-call device time (us): ``per_graph`` calls captured in one HIP graph, replayed
    ``iters`` times — removes host launch overhead, keeps the in-graph kernel boundaries that the
    real decode step also pays."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    ev[0].record()
    for i in range(iters):
        g.replay()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(iters))
    return ts[len(ts) // 2] * 1e3 / per_graph  # median us per call


def gemv_rows(C, dev, Ms=(1, 16, 32, 64, 128), sweep=True, grouped=False, shapes=None):
    """Cache-cold INT8 GEMV sweep.  ``grouped``: per-(token, 64-column) activation scales (the
    decode o/down projections after the fused producers)."""
    shapes = shapes or {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008),
                        "lm_head_int8": (32000, 4096)}
    out = []
    variants = [(0, 0, 0)]
    if sweep:
        variants += [(kw, u, ntw) for kw in (8, 16) for u in (2, 4) for ntw in (1, 2, 3, 4)]
    for name, (N, K) in shapes.items():
        # cache-cold: rotate through enough packed copies (> 1 GiB) that no call finds its weights
        # in the 256 MiB Infinity Cache — the decode regime, where 6.7 GB stream once per step
        ncopy = max(2, (1 << 30) // (N * K) + 1)
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
        sw = torch.rand(N, device=dev) * 0.01
        for M in Ms:
            if M > 64 and grouped and not C.rows128_ok(K, 1):
                continue                                  # (65-128 grouped rows: split-K shapes only)
            qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            sx = (torch.rand((K + 63) // 64, (M + 15) // 16 * 16, device=dev) if grouped
                  else torch.rand(M, device=dev)) * 0.01
            res = {}
            ctr = [0]

            def call():
                ctr[0] = (ctr[0] + 1) % ncopy
                return C.w8a8_gemm(qx, sx, wps[ctr[0]], sw, None, N, K)

            for rnd in range(2):  # interleaved rounds
                for nw, u, ntw in variants:
                    if (u == 4 and (M > 16 or ntw > 1)) or (M > 64 and (nw, u, ntw) != (0, 0, 0)):
                        continue
                    tune(C, "gemv", nw, u)
                    tune(C, "gemv_ntw", ntw, 0)
                    t = timeit(call, iters=10, per_graph=ncopy)
                    res.setdefault((nw, u, ntw), []).append(t)
            tune(C, "gemv", 0, 0)
            tune(C, "gemv_ntw", 0, 0)
            best = min(res, key=lambda k: min(res[k]))
            auto = min(res[(0, 0, 0)])
            nbytes = N * K + M * K + M * N * 2
            out.append(dict(op="w8a8_gemv" + ("_grouped" if grouped else ""), shape=name, M=M, N=N, K=K,
                            auto_us=round(auto, 2),
                            auto_TBps=round(nbytes / auto / 1e6, 2), best=list(best),
                            best_us=round(min(res[best]), 2), best_TBps=round(nbytes / min(res[best]) / 1e6, 2)))
            print(out[-1], flush=True)
    return out


def glu_rows(C, dev, Ms=(1, 16, 32, 64, 128)):
    """Decode MLP front half (Llama-2-7B: F = 11008), cache-cold: gate_up GEMV + SwiGLU writing
    bf16 h (2 or 4 tiles per workgroup) followed by the group-quant kernel, vs the 8-tile form
    that quantises h in its own epilogue (4 or 8 waves)."""
    out = []
    N, K = 2 * 11008, 4096
    ncopy = max(2, (1 << 30) // (N * K) + 1)
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
    wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
    sw = torch.rand(N, device=dev) * 0.01
    for M in Ms:
        qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        sx = torch.rand(M, device=dev) * 0.01
        ctr = [0]

        def bf16_then_quant():
            ctr[0] = (ctr[0] + 1) % ncopy
            return C.group_quant(C.w8a8_gemm_glu(qx, sx, wps[ctr[0]], sw, None, N, K))

        def quant_epilogue():
            ctr[0] = (ctr[0] + 1) % ncopy
            return C.w8a8_gemm_gluq(qx, sx, wps[ctr[0]], sw, None, N, K)

        variants = [("bf16+group_quant", bf16_then_quant, 0, 0)] if M <= 64 else []
        variants.append(("quant_epilogue", quant_epilogue, 0, 0))
        res = {}
        for rnd in range(2):
            for name, fn, ntw, nw in variants:
                tune(C, "gemv_ntw", ntw, 0)
                tune(C, "gemv", nw, 0)
                res.setdefault((name, ntw, nw), []).append(timeit(fn, iters=10, per_graph=ncopy))
        tune(C, "gemv_ntw", 0, 0)
        tune(C, "gemv", 0, 0)
        nbytes = N * K + M * K + M * N // 2
        for (name, ntw, nw), ts in res.items():
            out.append(dict(op="w8a8_glu", form=name, M=M, N=N, K=K, ntw=ntw, nw=nw, us=round(min(ts), 2),
                            TBps=round(nbytes / min(ts) / 1e6, 2)))
            print(out[-1], flush=True)
    return out


def other_rows(C, dev, only=None):
    want = lambda sec: only is None or sec in only  # noqa: E731
    out = []
    B, H, Hq, D = 16, 4096, 32, 128
    for L in ((256, 1024, 4096) if want("attn") else ()):
        S = L + 8
        q = torch.randn(B, Hq, D, device=dev).bfloat16()
        kc = torch.randn(B, Hq, S, D, device=dev).bfloat16()
        vc = torch.randn_like(kc)
        sl = torch.full((B,), L, dtype=torch.int32, device=dev)
        for tw in (256, 512, 1024):
            C.tune("decode_attn", tw, 0)
            t = timeit(lambda: C.decode_attn(q, kc, vc, sl, 1 / math.sqrt(D), L))
            nbytes = 2 * B * Hq * L * D * 2
            out.append(dict(op="decode_attn", B=B, Hkv=Hq, ctx=L, target_wg=tw, us=round(t, 2),
                            TBps=round(nbytes / t / 1e6, 2)))
            print(out[-1], flush=True)
        C.tune("decode_attn", 0, 0)
    for Bf, L in (((64, 160), (128, 160), (256, 150), (128, 512)) if want("attn_fused") else ()):
        # the model's decode attention: RoPE + KV append + attention + per-(token, 64) int8 output
        S = L + 8
        qkv = torch.randn(Bf, 3 * Hq * D, device=dev).bfloat16()
        kc = torch.randn(Bf, Hq, S, D, device=dev).bfloat16()
        vc = torch.randn_like(kc)
        sl = torch.full((Bf,), L, dtype=torch.int32, device=dev)
        rope = ops.rope_tables(D, S, 10000.0, device=dev)
        for occ, early in ((0, 1), (4, 0), (4, 1), (5, 0), (5, 1)):
            C.tune("decode_attn_occ", occ, 0)
            C.tune("decode_attn_early", early, 0)
            t = min(timeit(lambda: C.decode_attn_fused(qkv, sl - 1, rope, kc, vc, sl, Hq, 1 / math.sqrt(D), L, D,
                                                       True)) for _ in range(2))
            nbytes = 2 * Bf * Hq * L * D * 2
            out.append(dict(op="decode_attn_fused_q", B=Bf, Hkv=Hq, ctx=L, occ=occ, early=early, us=round(t, 2),
                            TBps=round(nbytes / t / 1e6, 2)))
            print(out[-1], flush=True)
        C.tune("decode_attn_occ", 4, 0)
        C.tune("decode_attn_early", 1, 0)
    if want("small"):
        out += small_rows(C, dev, B, H, Hq, D)
    if want("sample"):
        out += sample_rows(C, dev)
    if want("prefill"):
        out += prefill_rows(C, dev, Hq, D)
    for r in out[-12:]:
        print(r, flush=True)
    return out


def small_rows(C, dev, B, H, Hq, D):
    out = []
    x = torch.randn(B, H, device=dev).bfloat16()
    r = torch.randn(B, H, device=dev).bfloat16()
    w = torch.ones(H, device=dev).bfloat16()
    for rows in (B, 64):
        xx = torch.randn(rows, H, device=dev).bfloat16()
        rr = torch.randn(rows, H, device=dev).bfloat16()
        t = timeit(lambda: C.norm(xx, rr, w, None, 1e-5, True, True))
        out.append(dict(op="rmsnorm_res_quant", rows=rows, H=H, us=round(t, 2)))
    for rows, S in ((64, 4), (128, 4)):
        parts = torch.randn(S, rows, H, device=dev)
        rr = torch.randn(rows, H, device=dev).bfloat16()
        t = timeit(lambda: C.rms_norm_parts(parts, rr, w, 1e-5, True))
        out.append(dict(op="rmsnorm_parts_res_quant", rows=rows, S=S, H=H, us=round(t, 2)))
    gu = torch.randn(B, 2 * 11008, device=dev).bfloat16()
    out.append(dict(op="silu_mul_quant", rows=B, F=11008, us=round(timeit(lambda: C.act(gu, 0, True)), 2)))
    qkv = torch.randn(B, 3 * H, device=dev).bfloat16()
    kc = torch.zeros(B, Hq, 512, D, device=dev).bfloat16()
    vc = torch.zeros_like(kc)
    sp = torch.full((B,), 100, dtype=torch.int32, device=dev)
    rope = ops.rope_tables(D, 512, 10000.0, device=dev)
    out.append(dict(op="rope_kv_write", tokens=B, us=round(timeit(lambda: C.rope_kv_write(qkv, sp, rope, kc, vc, Hq, Hq, D, D)), 2)))
    return out


def sample_rows(C, dev):
    out = []
    rng = torch.tensor([1, 0], dtype=torch.int32, device=dev)
    for B, V in ((1, 32000), (16, 32000), (64, 32000), (128, 32000), (256, 32000), (16, 128256)):
        logits = (torch.randn(B, V, device=dev) * 3).bfloat16()
        seen = (torch.rand(B, V, device=dev) < 0.005).to(torch.uint8)
        for name, args in (("topk50_topp0.9", (0.7, 50, 0.9, 1.1, True)), ("greedy", (0.0, 0, 1.0, 1.1, False)),
                           ("full", (1.0, 0, 1.0, 1.0, True))):
            out.append(dict(op=f"sample_{name}", rows=B, V=V,
                            us=round(timeit(lambda: C.sample(logits, seen, *args, rng)), 2)))
            if name.startswith("topk"):       # split vs whole-row form (tune key sample_rowwide)
                for form, v in (("split", 0), ("rowwide", 1)):
                    C.tune("sample_rowwide", v, 0)
                    out[-1][f"{form}_us"] = round(timeit(lambda: C.sample(logits, seen, *args, rng)), 2)
                C.tune("sample_rowwide", 128, 0)
            if name.startswith("topk"):       # merge-kernel phase split (100 MHz wall clock)
                C.sample_timestamps(True)
                C.sample(logits, seen, *args, rng)
                torch.cuda.synchronize()
                ts = C.sample_timestamps(False)
                out[-1]["merge_phases_us"] = [round((ts[i + 1] - ts[i]) / 100.0, 2) for i in range(5)]
                out[-1]["merge_counts"] = [ts[8], ts[9]]
                out[-1]["chunk_phases_us"] = [round((ts[i + 1] - ts[i]) / 100.0, 2) for i in range(10, 13)]
                out[-1]["chunk_probes"] = ts[14]
            print(out[-1], flush=True)
    return out


def prefill_rows(C, dev, Hq, D):
    out = []
    # prefill attention (MFMA)
    D0 = D
    for T, Hkv, s0, D in ((512, Hq, 0, D0), (1024, Hq, 0, D0), (2048, Hq, 0, D0), (8192, Hq // 4, 0, D0),
                          (4096, Hq // 4, 28672, D0), (32768, Hq // 4, 0, D0), (1024, 8, 0, 64)):
        q = torch.randn(1, T, Hq, D, device=dev).bfloat16()
        kc = torch.randn(1, Hkv, s0 + T, D, device=dev).bfloat16()
        vc = torch.randn_like(kc)
        sp0 = torch.full((1,), s0, dtype=torch.int32, device=dev)
        flops = 4 * T * (s0 + T / 2) * D * Hq
        row = dict(op="prefill_attn_causal", T=T, start=s0, H=Hq, Hkv=Hkv, D=D)
        for name, v, stg in (("fa", 2, 2), ("fa_lockstep", 2, 1), ("old", 0, 0)):
            C.tune("prefill_fa", v, stg)
            t = timeit(lambda: C.prefill_attn(q, kc, vc, sp0, 1 / math.sqrt(D), True), iters=10,
                       per_graph=2 if T >= 16384 else 20)
            row[f"{name}_us"], row[f"{name}_TFLOPs"] = round(t, 2), round(flops / t / 1e6, 1)
        C.tune("prefill_fa", 1, 0)
        out.append(row)
        print(row, flush=True)
    return out


def batch1_rows(C, dev, M=1):
    """Batch-1 decode GEMVs at Llama-2-7B shapes, cache-cold: the quantising gate_up GEMV (8- vs
    16-wave workgroups) and the split-K o / down GEMVs over S slices (grouped activation scales)."""
    out = []
    N, K = 2 * 11008, 4096
    ncopy = max(2, (1 << 30) // (N * K) + 1)
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
    wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
    sw = torch.rand(N, device=dev) * 0.01
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
    sx = torch.rand(M, device=dev) * 0.01
    ctr = [0]

    def gluq():
        ctr[0] = (ctr[0] + 1) % ncopy
        return C.w8a8_gemm_gluq(qx, sx, wps[ctr[0]], sw, None, N, K)

    res = {}
    for rnd in range(3):
        for kw in (0, 8):
            tune(C, "gemv", kw, 0)
            res.setdefault(kw, []).append(timeit(gluq, iters=10, per_graph=ncopy))
    tune(C, "gemv", 0, 0)
    for kw, ts in res.items():
        out.append(dict(op="w8a8_gluq_m1", M=M, kw=kw, us=round(min(ts), 2), TBps=round(N * K / min(ts) / 1e6, 2)))
        print(out[-1], flush=True)
    del wps
    for name, (N, K) in {"o": (4096, 4096), "down": (4096, 11008)}.items():
        ncopy = max(2, (1 << 30) // (N * K) + 1)
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
        sw = torch.rand(N, device=dev) * 0.01
        qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        sx = torch.rand(K // 64, 16, device=dev) * 0.01
        res = {}
        for rnd in range(3):
            for S in (0, 1, 2, 4, 8):
                def call():
                    ctr[0] = (ctr[0] + 1) % ncopy
                    return C.w8a8_gemm_splitk(qx, sx, wps[ctr[0]], sw, None, N, K, S)
                res.setdefault(S, []).append(timeit(call, iters=10, per_graph=ncopy))
        for S, ts in res.items():
            out.append(dict(op="w8a8_splitk_m1", shape=name, M=M, S=S, us=round(min(ts), 2),
                            TBps=round(N * K / min(ts) / 1e6, 2)))
            print(out[-1], flush=True)
        del wps
    out += gemv_rows(C, dev, Ms=(M,), sweep=True, shapes={"qkv": (12288, 4096)})
    return out


def rows256_rows(C, dev, M=256):
    """One 256-row decode micro-batch (row-split ring2, weights read once) against two 128-row
    launches (the 2-lane form, weights read twice), cache-cold: qkv, o / down (grouped scales,
    split-K) and the quantising gate_up."""
    out = []
    shapes = {"qkv": (12288, 4096, "out"), "o": (4096, 4096, "part"), "gate_up": (22016, 4096, "gluq"),
              "down": (4096, 11008, "part"), "o_token": (4096, 4096, "part_tok"),
              "down_token": (4096, 11008, "part_tok")}
    for name, (N, K, kind) in shapes.items():
        ncopy = max(2, (1 << 30) // (N * K) + 1)
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
        sw = torch.rand(N, device=dev) * 0.01
        ctr = [0]

        def make(rows):
            qx = torch.randint(-127, 128, (rows, K), dtype=torch.int8, device=dev)
            sx = (torch.rand(K // 64, (rows + 15) // 16 * 16, device=dev) if kind == "part"
                  else torch.rand(rows, device=dev)) * 0.01

            def call():
                ctr[0] = (ctr[0] + 1) % ncopy
                if kind == "gluq":
                    return C.w8a8_gemm_gluq(qx, sx, wps[ctr[0]], sw, None, N, K)
                if kind in ("part", "part_tok"):
                    return C.w8a8_gemm_splitk(qx, sx, wps[ctr[0]], sw, None, N, K, 0)
                return C.w8a8_gemm(qx, sx, wps[ctr[0]], sw, None, N, K)
            return call

        c256, c128 = make(M), make(M // 2)
        res = {}
        for rnd in range(3):
            res.setdefault("r256", []).append(timeit(c256, iters=10, per_graph=ncopy))
            res.setdefault("two_x128", []).append(2 * timeit(c128, iters=10, per_graph=ncopy))
        row = dict(op="w8a8_rows256", shape=name, M=M, N=N, K=K, weight_MB=round(N * K / 1e6, 1))
        for form, ts in res.items():
            row[f"{form}_us"] = round(min(ts), 2)
            row[f"{form}_TBps"] = round(N * K / min(ts) / 1e6, 2)
        out.append(row)
        print(row, flush=True)
        del wps
    return out

def bf16_rows(C, dev, Ms=(8, 16, 32, 48, 64)):
    """bf16 decode projections at 1-64 rows (Llama-2-7B shapes), cache-cold: gemv_bf16.hip
    (1-4 row blocks of 16 per weight read) vs hipBLASLt through torch.nn.functional.linear."""
    out = []
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008),
              "lm_head": (32000, 4096)}
    for name, (N, K) in shapes.items():
        ncopy = max(2, (1 << 30) // (2 * N * K) + 1)
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(ncopy)]
        wps = [ops.pack_bf16_weight(w) for w in ws]
        for M in Ms:
            x = torch.randn(M, K, device=dev).bfloat16()
            ctr = [0]

            def ours():
                ctr[0] = (ctr[0] + 1) % ncopy
                return C.gemv_bf16(x, wps[ctr[0]], None, N, 0)

            def blas():
                ctr[0] = (ctr[0] + 1) % ncopy
                return torch.nn.functional.linear(x, ws[ctr[0]])

            t_o = min(timeit(ours, iters=10, per_graph=ncopy) for _ in range(2))
            t_b = min(timeit(blas, iters=10, per_graph=ncopy) for _ in range(2))
            out.append(dict(op="bf16_rows", shape=name, M=M, N=N, K=K, gemv_us=round(t_o, 2), hipblaslt_us=round(t_b, 2),
                            gemv_TBps=round(2 * N * K / t_o / 1e6, 2), hipblaslt_TBps=round(2 * N * K / t_b / 1e6, 2)))
            print(out[-1], flush=True)
        del ws, wps
    return out


def bf16_ring_rows(C, dev, Ms=(32, 64, 128, 256)):
    """bf16 decode projections at 17-256 rows (Llama-2-7B shapes), cache-cold: the bf16 ring GEMM
    (gemm_i8.hip ring2 kernel in bf16 operand mode) interleaved with
    hipBLASLt (torch.nn.functional.linear; gate_up + the SwiGLU kernel) and, up to 64 rows, the
    gemv_bf16.hip GEMV.  o / down are timed in their split-K form (fp32 slices for the norm)."""
    out = []
    shapes = {"qkv": (12288, 4096, 0), "o": (4096, 4096, 3), "gate_up": (22016, 4096, 1), "down": (4096, 11008, 3),
              "lm_head": (32000, 4096, 0)}
    for name, (N, K, epi) in shapes.items():
        ncopy = max(2, (1 << 30) // (2 * N * K) + 1)
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(ncopy)]
        wps = [ops.pack_bf16_weight(w) for w in ws]
        S = int(C.bf16_ring_splits(N, K)) if epi == 3 else 0
        for M in Ms:
            x = torch.randn(M, K, device=dev).bfloat16()
            ctr = [0]

            def ring():
                ctr[0] = (ctr[0] + 1) % ncopy
                return C.gemm_bf16_ring(x, wps[ctr[0]], None, N, epi, S)

            def blas():
                ctr[0] = (ctr[0] + 1) % ncopy
                y = torch.nn.functional.linear(x, ws[ctr[0]])
                return ops.activation(y, "silu_glu") if epi == 1 else y

            def gemv():
                ctr[0] = (ctr[0] + 1) % ncopy
                return C.gemv_bf16(x, wps[ctr[0]], None, N, 1 if epi == 1 else 0)

            res = {}
            for _ in range(2):
                res.setdefault("ring", []).append(timeit(ring, iters=10, per_graph=ncopy))
                res.setdefault("hipblaslt", []).append(timeit(blas, iters=10, per_graph=ncopy))
                if M <= 64:
                    res.setdefault("gemv", []).append(timeit(gemv, iters=10, per_graph=ncopy))
            row = dict(op="bf16_ring", shape=name, M=M, N=N, K=K, S=S)
            for k, ts in res.items():
                row[k + "_us"] = round(min(ts), 2)
                row[k + "_TBps"] = round(2 * N * K / min(ts) / 1e6, 2)
            out.append(row)
            print(row, flush=True)
        del ws, wps
    return out


def knob_ab_rows(C, dev, knob, values=(1, 0), M=256, shapes=None):
    """A/B of one tuning knob (``tune knob=v``) on the 256-row decode GEMMs, interleaved rounds,
    cache-cold weights; also checks that every setting gives the same output bits as the first."""
    out = []
    shapes = shapes or {"qkv": (12288, 4096, "out"), "gate_up": (22016, 4096, "gluq"), "o": (4096, 4096, "part"),
                        "down": (4096, 11008, "part")}
    for name, (N, K, kind) in shapes.items():
        ncopy = max(2, (1 << 30) // (N * K) + 1)
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wps = [ops.pack_int8_weight(w) for _ in range(ncopy)]
        sw = torch.rand(N, device=dev) * 0.01
        qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        sx = (torch.rand(K // 64, (M + 15) // 16 * 16, device=dev) if kind == "part" else torch.rand(M, device=dev)) * 0.01
        ctr = [0]

        def call(wp=None):
            if wp is None:
                ctr[0] = (ctr[0] + 1) % ncopy
                wp = wps[ctr[0]]
            if kind == "gluq":
                return C.w8a8_gemm_gluq(qx, sx, wp, sw, None, N, K)
            if kind == "part":
                return C.w8a8_gemm_splitk(qx, sx, wp, sw, None, N, K, 0)
            return C.w8a8_gemm(qx, sx, wp, sw, None, N, K)
        res, same = {}, True
        ref = None
        for v in values:
            C.tune(knob, v, 0)
            o = call(wps[0])
            o = [x.clone() for x in o] if isinstance(o, (tuple, list)) else [o.clone()]
            if ref is None:
                ref = o
            else:
                same = same and all(torch.equal(a, b) for a, b in zip(ref, o))
        for _ in range(3):
            for v in values:
                C.tune(knob, v, 0)
                res.setdefault(v, []).append(timeit(call, iters=10, per_graph=ncopy))
        C.tune(knob, values[0], 0)
        row = dict(op=f"ab_{knob}", shape=name, M=M, N=N, K=K, identical=bool(same))
        for v, ts in res.items():
            row[f"{knob}{v}_us"] = round(min(ts), 2)
        out.append(row)
        print(row, flush=True)
        del wps
    return out


def x32_rows(C, dev, Ms=(2048, 16384)):
    """Prefill INT8 GEMM: the 256 x 256 v_mfma_i32_32x32x32_i8 kernel (tune prefill_x32 2: from 192
    tiles) against the 128 x 256 16x16x64 kernel (prefill_x32 0), interleaved, Llama-2-7B shapes."""
    out = []
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008)}
    for name, (N, K) in shapes.items():
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        wp = ops.pack_int8_weight(w)
        s2 = torch.rand(N, device=dev) * 0.01
        for M in Ms:
            a = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            s1 = torch.rand(M, device=dev) * 0.01
            res = {}
            per = max(2, min(20, int(4e11 // (M * N * K))))
            for _ in range(3):
                for v in (0, 2):
                    C.tune("prefill_x32", v, 0)
                    res.setdefault(v, []).append(timeit(lambda: C.w8a8_gemm(a, s1, wp, s2, None, N, K), iters=5,
                                                        per_graph=per))
            C.tune("prefill_x32", 1, 0)
            row = dict(op="w8a8_gemm_prefill_x32", shape=name, M=M, N=N, K=K)
            for v, ts in res.items():
                row[f"x32_{v}_us"] = round(min(ts), 1)
                row[f"x32_{v}_TOPs"] = round(2 * M * N * K / min(ts) / 1e6, 1)
            out.append(row)
            print(row, flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-sweep", action="store_true")
    ap.add_argument("--tune", action="append", default=[], help="name=a[,b] passed to ext().tune (repeatable)")
    ap.add_argument("--only", default=None, help="comma list of: gemv,grouped,glu,attn,attn_fused,small,sample,prefill,pgemm,m1,ring")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else None
    dev = torch.device("cuda:0")
    C = ops.ext()
    for t in a.tune:
        name, vals = t.split("=")
        v = [int(x) for x in vals.split(",")] + [0]
        GLOBAL_TUNE.append((name, v[0], v[1]))
        C.tune(name, v[0], v[1])
    rows = gemv_rows(C, dev, sweep=not a.no_sweep) if only is None or "gemv" in only else []
    if only is None or "grouped" in only:
        rows += gemv_rows(C, dev, sweep=not a.no_sweep, grouped=True,
                          shapes={"o": (4096, 4096), "down": (4096, 11008)})
    if only is None or "glu" in only:
        rows += glu_rows(C, dev)
    rows += other_rows(C, dev, only)
    if only is not None and "m1" in only:
        rows += batch1_rows(C, dev)
    if only is not None and "rows256" in only:
        rows += rows256_rows(C, dev)
    if only is not None and "bf16rows" in only:
        rows += bf16_rows(C, dev)
    if only is not None and "x32" in only:
        rows += x32_rows(C, dev)
    if only is not None and "bf16ring" in only:
        rows += bf16_ring_rows(C, dev)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()

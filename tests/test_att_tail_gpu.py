"""Batch-1 decode with the attention in the qkv GEMV's tail (ops.w8a8_gemv_norm_att, gemm_i8.hip
att_tail): norm prologue -> W8A8 qkv GEMV -> RoPE + KV append + attention of each KV-head group
by the workgroup that completes the group's tiles -> per-(token, 64) int8 for the o projection.

Checked against the unfused launches (norm-prologue GEMV, then the split-K decode attention with
int8 output) and the fp32 reference composition; the KV append, the residual rows, the arrival
counters (zero after every launch), run-to-run determinism, and a Llama decoder / Generator at
batch 1 (graph-captured) with the tail on and off."""
import math

import pytest
import torch

from edgellm import ops
from edgellm.models.layers import PendingNorm
from edgellm.ops import _ref

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    bad = (err > atol + rtol * b.abs()).sum().item()
    assert bad == 0, f"{bad} / {a.numel()} elements off, max err {err.max().item():.4g}"


# Llama-2-7B (G 1, D 128), Llama-3.2-1B (G 4, D 64), a G 4 / D 128 geometry (Llama-3-8B-like)
@pytest.mark.parametrize("Hq,Hkv,D,K", [(32, 32, 128, 4096), (32, 8, 64, 2048), (16, 4, 128, 2048),
                                         (32, 8, 128, 4096)])
@pytest.mark.parametrize("S", [1, 2, 4])
@pytest.mark.parametrize("ln", [1, 2, 17, 300, 1024])
def test_att_tail_matches_unfused(cuda, Hq, Hkv, D, K, S, ln):
    torch.manual_seed(Hq + D + K + S + ln)
    rot, eps = D, 1e-5
    N = (Hq + 2 * Hkv) * D
    parts = torch.randn(S, 1, K, device=cuda) * 0.5
    res = torch.randn(1, K, device=cuda).bfloat16()
    gamma = (torch.rand(K, device=cuda) + 0.5).bfloat16()
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    wp = ops.pack_int8_weight(w)
    sw = torch.rand(N, device=cuda) * 0.002 + 1e-4
    bias = torch.randn(N, device=cuda).bfloat16() if S == 2 else None
    Smax = max(ln + 3, 64)
    kc = torch.randn(1, Hkv, Smax, D, device=cuda).bfloat16()
    vc = torch.randn(1, Hkv, Smax, D, device=cuda).bfloat16()
    kr, vr = kc.clone(), vc.clone()
    sl = torch.tensor([ln], dtype=torch.int32, device=cuda)
    pos = sl - 1
    rope = ops.rope_tables(rot, Smax, 10000.0, device=cuda)
    scale = 1 / math.sqrt(D)

    # unfused: norm-prologue GEMV, then the decode attention launch with int8 output
    h_ref = torch.empty(1, K, device=cuda).bfloat16()
    y = ops.w8a8_gemv_norm(parts, res, gamma, eps, h_ref, wp, sw, bias, N, K)
    assert y is not None
    uq, us = ops.decode_attention_fused(y, pos, rope, kr, vr, sl, Hq, scale, ln, rot, True)
    # fp32 reference of the attention over the same qkv row
    kf, vf = kc.clone(), vc.clone()
    q = _ref.rope_kv_write(y, pos, rope, kf, vf, Hq, Hkv, D, rot)
    ref = _ref.decode_attention(q.view(1, Hq, D), kf, vf, sl, scale).reshape(1, Hq * D).float()

    h = torch.full((1, K), float("nan"), device=cuda).bfloat16()
    r = ops.w8a8_gemv_norm_att(PendingNorm(parts, res, gamma, eps, h), wp, sw, bias, K, kc, vc, pos, sl, rope, rot,
                               Hq, scale, ln)
    assert r is not None
    fq, fs = r
    assert fq.shape == (1, Hq * D) and fs.shape == (Hq * D // 64, 16)
    assert torch.equal(h, h_ref), "residual rows differ from the norm prologue's"
    assert torch.equal(vc, vr), "value append differs"
    _close(kc, kr, 1e-2, 1e-2)                          # RoPE'd key: same formula, fp32 contraction may differ
    cnt = ops._att_counters(kc[:1], Hkv)
    assert int(cnt.abs().sum()) == 0, "arrival counters not restored"
    deq = fq.float() * fs[:, :1].t().repeat_interleave(64, 1)
    udeq = uq.float() * us[:, :1].t().repeat_interleave(64, 1)
    # int8 output: within one quantisation step of its group (+ the attention's bf16 rounding)
    step = fs[:, :1].t().repeat_interleave(64, 1).cpu()
    for a, b in ((deq, ref), (deq, udeq)):
        err = (a.cpu() - b.cpu()).abs()
        bad = (err > 1.01 * step + 1e-2 * b.abs().cpu() + 1e-3).sum().item()
        assert bad == 0, f"{bad} elements beyond one int8 step, max err {err.max().item():.4g}"

    # run-to-run: the same launch over the same inputs is bit-identical
    kc2, vc2 = kr.clone(), vr.clone()
    kc2[:, :, ln - 1] = kr[:, :, ln - 1] * 0 + 7      # overwritten by the append
    r2 = ops.w8a8_gemv_norm_att(PendingNorm(parts, res, gamma, eps, torch.empty_like(h)), wp, sw, bias, K, kc2, vc2,
                                pos, sl, rope, rot, Hq, scale, ln)
    assert torch.equal(r2[0], fq) and torch.equal(r2[1][:, :1], fs[:, :1])
    assert torch.equal(kc2, kc)


def test_att_tail_declines(cuda, monkeypatch):
    """Geometries without an instantiation, long caches and the off knob return None."""
    K, Hq, Hkv, D = 4096, 32, 32, 128
    N = (Hq + 2 * Hkv) * D
    wp = ops.pack_int8_weight(torch.zeros(N, K, dtype=torch.int8, device=cuda))
    sw = torch.ones(N, device=cuda)
    pn = PendingNorm(torch.zeros(2, 1, K, device=cuda), torch.zeros(1, K, device=cuda).bfloat16(),
                     torch.ones(K, device=cuda).bfloat16(), 1e-5, torch.empty(1, K, device=cuda).bfloat16())
    kc = torch.zeros(1, Hkv, 64, D, device=cuda).bfloat16()
    sl = torch.tensor([5], dtype=torch.int32, device=cuda)
    rope = ops.rope_tables(D, 64, 10000.0, device=cuda)
    args = (pn, wp, sw, None, K, kc, kc.clone(), sl - 1, sl, rope, D, Hq, 0.1)
    assert ops.w8a8_gemv_norm_att(*args, 5) is not None
    assert ops.w8a8_gemv_norm_att(*args, ops.ATT_TAIL_MAX_LEN + 1) is None
    monkeypatch.setattr(ops, "ATT_TAIL_MAX_LEN", 0)
    assert ops.w8a8_gemv_norm_att(*args, 5) is None
    monkeypatch.undo()
    # G = 2 has no instantiation
    Hkv2 = 16
    N2 = (Hq + 2 * Hkv2) * D
    wp2 = ops.pack_int8_weight(torch.zeros(N2, K, dtype=torch.int8, device=cuda))
    kc2 = torch.zeros(1, Hkv2, 64, D, device=cuda).bfloat16()
    assert ops.w8a8_gemv_norm_att(pn, wp2, torch.ones(N2, device=cuda), None, K, kc2, kc2.clone(), sl - 1, sl, rope,
                                  D, Hq, 0.1, 5) is None


@pytest.mark.parametrize("heads,kv_heads,D", [(16, 4, 128), (16, 16, 128), (32, 8, 64)])
def test_llama_batch1_decode_att_tail(cuda, heads, kv_heads, D, monkeypatch):
    """A W8A8 Llama decoder at batch 1: decode steps with the tail == with the separate attention
    launch up to the attention's rounding (logits), the caches likewise; and the Generator (graph
    captured, greedy) produces the same tokens graph-replayed and eager with the tail on."""
    from edgellm.engine import Generator, KVCache, SamplingParams
    from edgellm.models import AttnCtx, build_model, tiny
    from edgellm.quant import quantize_model
    cfg = tiny("llama", hidden_size=2048, num_heads=heads, num_kv_heads=kv_heads, head_dim=D, rotary_dim=D,
               intermediate_size=4096, num_layers=3)
    qm = quantize_model(build_model(cfg, device=cuda, seed=5), "w8a8")
    T = 9
    ids = torch.randint(0, cfg.vocab_size, (1, T), generator=torch.Generator().manual_seed(1)).to(cuda)
    calls = []
    orig = ops.w8a8_gemv_norm_att

    def spy(*a, **k):
        r = orig(*a, **k)
        calls.append(r is not None)
        return r

    monkeypatch.setattr(ops, "w8a8_gemv_norm_att", spy)
    outs, caches = [], []
    for cap in (ops.ATT_TAIL_MAX_LEN, 0):
        monkeypatch.setattr(ops, "ATT_TAIL_MAX_LEN", cap)
        kv = KVCache(cfg, 1, T + 8, dtype=qm.dtype, device=cuda)
        sp0 = torch.zeros(1, dtype=torch.int32, device=cuda)
        logits = []
        with torch.no_grad():
            qm(ids, AttnCtx("prefill", 1, T, sp0, sp0 + T, T, kv.rows(0, 1), qm.rope_table(cuda)), logits="last")
            tok = ids[:, -1:]
            for s in range(4):
                pos = torch.full((1,), T + s, dtype=torch.int32, device=cuda)
                lg = qm(tok, AttnCtx("decode", 1, 1, pos, pos + 1, T + s + 1, kv.rows(0, 1), qm.rope_table(cuda)))
                logits.append(lg.float().reshape(-1))
                tok = ids[:, s:s + 1]                          # teacher-forced: both runs see the same tokens
        outs.append(torch.stack(logits))
        caches.append(kv.layer(1)[0][:, :, :T + 4].float().clone())
    n = len(calls) // 2                                  # layers 1.. at each decode step, tail on then off
    assert n > 0 and all(calls[:n]) and not any(calls[n:]), calls
    cos = torch.nn.functional.cosine_similarity(outs[0], outs[1], dim=-1)
    assert cos.min().item() > 0.999, cos
    _close(caches[0], caches[1], 2e-2, 2e-2)

    monkeypatch.setattr(ops, "ATT_TAIL_MAX_LEN", 1024)
    sp = SamplingParams(max_new_tokens=24, do_sample=False)
    prompt = ids[0].tolist()
    g_graph = Generator(qm, max_batch=1, max_seq=64)
    a = g_graph.generate([prompt], sp).tokens
    assert g_graph._graphs, "decode did not run graph-captured"
    b = Generator(qm, max_batch=1, max_seq=64, use_graphs=False).generate([prompt], sp).tokens
    assert a == b
    c = g_graph.generate([prompt], sp).tokens            # replay again: counters were left at zero
    assert c == a

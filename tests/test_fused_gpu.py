"""Fused decode-path kernels vs the fp32 reference composition of the unfused ops.

* decode attention straight from the QKV projection (RoPE + KV append + attention, optional
  per-group int8 output) == ops._ref rope_kv_write -> decode_attention (-> quant_per_group)
* W8A8 GEMV with per-(token, 64-column) activation scales == _ref.w8a8_linear (2-D x_scale)
* gate_up GEMV + SwiGLU epilogue (16-blocked rows) == _ref composition; per-(token, 64) group
  quantisation kernel == _ref.quant_per_group
* blocked-layout activation kernel (prefill path of the same packing)
"""
import math

import pytest
import torch

from edgellm import ops
from edgellm.ops import _ref

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    bad = (err > atol + rtol * b.abs()).sum().item()
    assert bad == 0, f"{bad} / {a.numel()} elements off, max err {err.max().item():.4g}"


@pytest.mark.parametrize("Hq,Hkv,D,rot", [(32, 32, 128, 128), (32, 8, 128, 128), (32, 8, 64, 64), (32, 32, 80, 32),
                                          (8, 8, 256, 64), (12, 12, 64, 0)])
@pytest.mark.parametrize("lens", [(1, 17, 200), (4096, 1000, 3333), (200,), (513,)])
@pytest.mark.parametrize("quant", [False, True])
@pytest.mark.parametrize("occ", [0, 4, 5])
def test_decode_attention_fused(cuda, Hq, Hkv, D, rot, lens, quant, occ):
    """(one sequence: MHA grids below decode_attn_small workgroups take the double-buffered form
    under the default occ 4)"""
    if quant and D % 64:
        pytest.skip("per-group output needs D % 64 == 0")
    C = ops.ext()
    C.tune("decode_attn_occ", occ, 0)
    try:
        _check_decode_attention_fused(C, Hq, Hkv, D, rot, lens, quant)
    finally:
        C.tune("decode_attn_occ", 4, 0)


@pytest.mark.parametrize("lens", [(1, 17, 200), (150, 151, 152, 149), (4096, 1000, 3333), (513, 60), (127, 128, 129)])
@pytest.mark.parametrize("quant", [False, True])
@pytest.mark.parametrize("unroll", [4, 8])
def test_decode_attention_fused_unroll(cuda, lens, quant, unroll):
    """The barrier-free MHA D = 128 form (the bench's attention) with 4 or 8 key groups per wave
    per chunk (tune decode_attn_unroll; 8 skips the loads of groups past the end)."""
    C = ops.ext()
    C.tune("decode_attn_unroll", unroll, 0)
    try:
        _check_decode_attention_fused(C, 32, 32, 128, 128, lens, quant)
    finally:
        C.tune("decode_attn_unroll", 4, 0)


@pytest.mark.parametrize("Hq,Hkv,D,rot", [(32, 32, 128, 128), (32, 32, 80, 32), (8, 8, 256, 64), (12, 12, 64, 0),
                                          (32, 8, 64, 64), (32, 8, 128, 128)])
@pytest.mark.parametrize("lens", [(1,), (200,), (255, 3), (300,), (700,)])
@pytest.mark.parametrize("small", [64, 0])
@pytest.mark.parametrize("quant", [False, True])
def test_decode_attention_small_grid_forms(cuda, Hq, Hkv, D, rot, lens, small, quant):
    """Small grids: the double-buffered form MHA grids below 64 workgroups take by default
    (decode_attn_small 64) and the single-buffered form (0 = routing off) against the reference;
    GQA grids keep the query-head split either way."""
    if quant and D % 64:
        pytest.skip("per-group output needs D % 64 == 0")
    C = ops.ext()
    C.tune("decode_attn_small", small, 0)
    try:
        # (255,): one rotated key element lands within 1e-8 of zero, where the kernel's and torch's
        # fp32 contractions round to different bf16 values: the cache is checked to 1 bf16 ulp there
        _check_decode_attention_fused(C, Hq, Hkv, D, rot, lens, quant, exact_cache=False)
    finally:
        C.tune("decode_attn_small", 64, 0)


@pytest.mark.parametrize("Hq,Hkv,D,rot", [(32, 8, 64, 64), (32, 8, 128, 128), (16, 2, 128, 64), (8, 4, 256, 64)])
@pytest.mark.parametrize("lens", [(1, 17, 200), (4096, 1000, 3333), (300,)])
@pytest.mark.parametrize("gsplit", [1, 2])
@pytest.mark.parametrize("quant", [False, True])
def test_decode_attention_gsplit(cuda, Hq, Hkv, D, rot, lens, gsplit, quant):
    """Query-head split (one workgroup per query head, the new key rebuilt in every workgroup of a
    KV head, stored by the first): forced on (2) and off (1), fused append + output quant, and the
    plain kernel."""
    C = ops.ext()
    C.tune("decode_attn_gsplit", gsplit, 0)
    try:
        _check_decode_attention_fused(C, Hq, Hkv, D, rot, lens, quant)
        B = len(lens)
        S = max(lens) + 5
        q = torch.randn(B, Hq, D, device=cuda).bfloat16()
        kc = torch.randn(B, Hkv, S, D, device=cuda).bfloat16()
        vc = torch.randn(B, Hkv, S, D, device=cuda).bfloat16()
        sl = torch.tensor(lens, device=cuda, dtype=torch.int32)
        _close(C.decode_attn(q, kc, vc, sl, 1 / math.sqrt(D), S), _ref.decode_attention(q, kc, vc, sl, 1 / math.sqrt(D)),
               2e-2, 2e-2)
    finally:
        C.tune("decode_attn_gsplit", 0, 0)


def _check_decode_attention_fused(C, Hq, Hkv, D, rot, lens, quant, exact_cache=True):
    cuda = torch.device("cuda")
    torch.manual_seed(3)
    B = len(lens)
    S = max(lens) + 5
    W = (Hq + 2 * Hkv) * D
    qkv = torch.randn(B, W, device=cuda).bfloat16()
    kc = torch.randn(B, Hkv, S, D, device=cuda).bfloat16()
    vc = torch.randn(B, Hkv, S, D, device=cuda).bfloat16()
    kr, vr = kc.clone(), vc.clone()
    sl = torch.tensor(lens, device=cuda, dtype=torch.int32)
    pos = sl - 1
    rope = ops.rope_tables(rot, S, 10000.0, device=cuda) if rot else None
    scale = 1 / math.sqrt(D)
    out, s = C.decode_attn_fused(qkv, pos, rope, kc, vc, sl, Hq, scale, max(lens), rot, quant)
    q = _ref.rope_kv_write(qkv, pos, rope, kr, vr, Hq, Hkv, D, rot)
    ref = _ref.decode_attention(q.view(B, Hq, D), kr, vr, sl, scale)
    if exact_cache:
        assert torch.equal(kc, kr) and torch.equal(vc, vr), "KV append differs from rope_kv_write"
    else:
        assert torch.equal(vc, vr), "V append differs"
        _close(kc, kr, 1e-6, 1 / 128)
    if quant:
        qr, sr = _ref.quant_per_group(ref.reshape(B, Hq * D))
        deq = out.float() * s[:, :B].t().repeat_interleave(64, 1)
        _close(deq, ref.reshape(B, -1), 3e-2, 3e-2)
        _close(s[:, :B], sr[:, :B], 1e-3, 2e-2)
    else:
        _close(out, ref, 2e-2, 2e-2)


@pytest.mark.parametrize("M", [1, 2, 5, 16, 33, 64])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (1040, 128), (22016, 4096)])
def test_w8a8_gemm_group_scales(cuda, M, N, K):
    C = ops.ext()
    torch.manual_seed(M)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    mpad = (M + 15) // 16 * 16
    sx = torch.rand(K // 64, mpad, device=cuda) * 0.02 + 1e-3
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.02 + 1e-3
    bias = torch.randn(N, device=cuda).bfloat16()
    out = C.w8a8_gemm(qx, sx, ops.pack_int8_weight(w), sw, bias, N, K)
    _close(out, _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32), 1e-2, 1e-2)


@pytest.mark.parametrize("M", [1, 3, 16, 40, 64])
@pytest.mark.parametrize("F,K", [(1024, 4096), (11008, 4096), (256, 128)])
def test_w8a8_glu_fused(cuda, M, F, K):
    """gate_up GEMV on 16-blocked rows with the SwiGLU epilogue == unfused GEMM -> silu(g) * u."""
    C = ops.ext()
    torch.manual_seed(F + M)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.004 + 1e-4
    w = torch.randint(-127, 128, (2 * F, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(2 * F, device=cuda) * 0.004 + 1e-4
    wb, swb = _ref.block_glu_rows(w), _ref.block_glu_rows(sw)
    h = C.w8a8_gemm_glu(qx, sx, ops.pack_int8_weight(wb), swb, None, 2 * F, K)
    y = _ref.w8a8_linear(qx, sx, w, sw, None, torch.bfloat16)               # unblocked [gate | up], bf16
    ref = _ref.silu_mul(y)
    assert h.shape == (M, F) and h.dtype == torch.bfloat16
    # g and u are bf16-rounded on both sides; float-vs-double products can land 1 ulp apart
    _close(h, ref, 1e-3, 2e-2)


@pytest.mark.parametrize("M", [1, 16, 33, 64])
@pytest.mark.parametrize("F,K", [(64, 64), (192, 4096), (11008, 4096)])
def test_w8a8_glu_quant_epilogue(cuda, M, F, K):
    """gate_up GEMV + SwiGLU + per-(token, 64 features) int8 quantisation in one kernel ==
    unfused GEMM -> silu(g) * u -> quant_per_group (fp32 h on both sides)."""
    C = ops.ext()
    torch.manual_seed(F + M + 7)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.004 + 1e-4
    w = torch.randint(-127, 128, (2 * F, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(2 * F, device=cuda) * 0.004 + 1e-4
    wb, swb = _ref.block_glu_rows(w), _ref.block_glu_rows(sw)
    q, s = C.w8a8_gemm_gluq(qx, sx, ops.pack_int8_weight(wb), swb, None, 2 * F, K)
    g, u = _ref.w8a8_linear(qx, sx, w, sw, None, torch.bfloat16).float().chunk(2, dim=-1)
    qr, sr = _ref.quant_per_group(torch.nn.functional.silu(g) * u)
    assert q.shape == (M, F) and q.dtype == torch.int8 and s.shape == sr.shape
    _close(s, sr, 1e-7, 1e-5)
    assert (s[:, M:] == 0).all()
    assert (q.int() - qr.int()).abs().max().item() <= 1


@pytest.mark.parametrize("M", [1, 5, 16, 64])
@pytest.mark.parametrize("K", [64, 4096, 11008])
def test_group_quant(cuda, M, K):
    C = ops.ext()
    x = (torch.randn(M, K, device=cuda) * 3).bfloat16()
    q, s = C.group_quant(x)
    qr, sr = _ref.quant_per_group(x)
    _close(s[:, :M], sr[:, :M], 1e-7, 1e-5)
    assert (q.int() - qr.int()).abs().max().item() <= 1


@pytest.mark.parametrize("F", [256, 11008])
def test_act_blocked_glu(cuda, F):
    C = ops.ext()
    x = torch.randn(5, 2 * F, device=cuda).bfloat16() * 2
    y, _ = C.act(x, 3, False)
    _close(y, _ref.silu_mul(_ref.unblock_glu(x)), 2e-2, 1e-2)
    q, s = C.act(x, 3, True)
    qr, sr = _ref.silu_mul_quant(_ref.unblock_glu(x))
    _close(s, sr, 0, 2e-3)
    assert (q.int() - qr.int()).abs().max().item() <= 1


@pytest.mark.parametrize("cfg", [(0, 0, 0), (8, 2, 1), (16, 4, 1), (16, 2, 2), (16, 2, 3), (8, 2, 4)])
@pytest.mark.parametrize("grouped", [False, True])
@pytest.mark.parametrize("M,N,K", [(16, 4096, 4096), (7, 12288, 4096), (40, 4096, 11008), (16, 1040, 1024),
                                   (64, 1056, 4096), (33, 12288, 4096)])
def test_gemv_configs(cuda, cfg, grouped, M, N, K):
    """Every (k-waves, unroll, tiles-per-workgroup) variant of the weight-stationary GEMV gives the
    reference answer, and repeated launches are bit-identical (deterministic LDS reduction)."""
    C = ops.ext()
    torch.manual_seed(sum(cfg) + M)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = (torch.rand(K // 64, (M + 15) // 16 * 16, device=cuda) if grouped else torch.rand(M, device=cuda)) * 0.02
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.02 + 1e-3
    wp = ops.pack_int8_weight(w)
    try:
        C.tune("gemv", cfg[0], cfg[1])
        C.tune("gemv_ntw", cfg[2], 0)
        outs = [C.w8a8_gemm(qx, sx, wp, sw, None, N, K) for _ in range(2)]
    finally:
        C.tune("gemv", 0, 0)
        C.tune("gemv_ntw", 0, 0)
    assert torch.equal(outs[0], outs[1])
    _close(outs[0], _ref.w8a8_linear(qx, sx, w, sw, None, torch.float32), 1e-2, 1e-2)


@pytest.mark.parametrize("M", [1, 16, 17, 40, 64])
def test_glu_forms_agree(cuda, M):
    """bf16-h GLU and the quantising GLU epilogue agree with the reference for 1..4 row blocks."""
    C = ops.ext()
    F, K = 11008, 4096
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.004 + 1e-4
    w = torch.randint(-127, 128, (2 * F, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(2 * F, device=cuda) * 0.004 + 1e-4
    wb, swb = _ref.block_glu_rows(w), _ref.block_glu_rows(sw)
    wp = ops.pack_int8_weight(wb)
    h = C.w8a8_gemm_glu(qx, sx, wp, swb, None, 2 * F, K)
    y = _ref.w8a8_linear(qx, sx, wb, swb, None, torch.bfloat16)
    ref = _ref.silu_mul(_ref.unblock_glu(y))
    _close(h, ref, 2e-2, 2e-2)
    q, s = C.w8a8_gemm_gluq(qx, sx, wp, swb, None, 2 * F, K)
    step = s[:, :M].t().unsqueeze(-1)                                    # [M, F/64, 1]
    deq = q.float().view(M, F // 64, 64) * step
    err = (deq - ref.float().view(M, F // 64, 64)).abs()
    assert (err <= 0.51 * step + 1e-2 * ref.float().view(M, F // 64, 64).abs() + 1e-3).all(), err.max().item()


@pytest.mark.parametrize("M", [65, 100, 128])
@pytest.mark.parametrize("grouped", [False, True])
@pytest.mark.parametrize("N,K,S", [(12288, 4096, 1), (4096, 4096, 4), (4096, 11008, 4), (1024, 14336, 4)])
def test_gemv_rows128(cuda, M, grouped, N, K, S):
    """65-128 rows (ring2 kernel, 8 row blocks): whole-K outputs and split-K partial slices against
    the fp32 reference, per-token and per-(token, 64) activation scales."""
    C = ops.ext()
    assert C.rows128_ok(K, S)
    torch.manual_seed(M + K)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = (torch.rand(K // 64, (M + 15) // 16 * 16, device=cuda) if grouped else torch.rand(M, device=cuda)) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    if S == 1:
        out = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        _close(out, ref, 1e-2, 1e-2)
    else:
        parts = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, S)
        assert parts.shape == (S, M, N)
        _close(parts.sum(0), ref, 1e-3, 1e-2)
        assert torch.equal(parts, C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, S))


@pytest.mark.parametrize("M", [65, 100, 128])
def test_gluq_beyond_64_rows(cuda, M):
    """The quantising GLU epilogue at 5-8 row blocks (ring2 kernel, K = 4096)."""
    C = ops.ext()
    F, K = 11008, 4096
    torch.manual_seed(M)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.004 + 1e-4
    w = torch.randint(-127, 128, (2 * F, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(2 * F, device=cuda) * 0.004 + 1e-4
    wb, swb = _ref.block_glu_rows(w), _ref.block_glu_rows(sw)
    wp = ops.pack_int8_weight(wb)
    ref = _ref.silu_mul(_ref.unblock_glu(_ref.w8a8_linear(qx, sx, wb, swb, None, torch.bfloat16)))
    q, s = C.w8a8_gemm_gluq(qx, sx, wp, swb, None, 2 * F, K)
    step = s[:, :M].t().unsqueeze(-1)
    deq = q.float().view(M, F // 64, 64) * step
    err = (deq - ref.float().view(M, F // 64, 64)).abs()
    assert (err <= 0.51 * step + 1e-2 * ref.float().view(M, F // 64, 64).abs() + 1e-3).all(), err.max().item()


@pytest.mark.parametrize("M", [1, 7, 16, 32, 64])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (2048, 8192), (1040, 1024)])
@pytest.mark.parametrize("grouped", [False, True])
def test_gemv_split_k_partials(cuda, M, N, K, grouped):
    """Split-K partial slices: their in-order sum equals the unsplit GEMV (fp32 tolerance), and
    the bf16 rounding of that sum equals the unsplit bf16 output to one ulp."""
    C = ops.ext()
    torch.manual_seed(M + N)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = (torch.rand(K // 64, (M + 15) // 16 * 16, device=cuda) if grouped else torch.rand(M, device=cuda)) * 0.02
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.02 + 1e-3
    bias = torch.randn(N, device=cuda).bfloat16()
    wp = ops.pack_int8_weight(w)
    parts = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, 0)
    assert parts.dim() == 3 and parts.shape[1:] == (M, N) and 1 <= parts.shape[0] <= 8
    from edgellm.models.layers import PartialSum
    y = PartialSum(parts).materialize()
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    _close(parts.sum(0), ref, 1e-2, 1e-4)
    _close(y, C.w8a8_gemm(qx, sx, wp, sw, bias, N, K), 1e-2, 1e-2)
    assert torch.equal(C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, 0), parts)     # deterministic


@pytest.mark.parametrize("M", [1, 16, 40])
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("quant", [False, True])
def test_rms_norm_parts(cuda, M, with_res, quant):
    """Norm over split-K slices == norm over the materialised bf16 sum (the same kernel math)."""
    from edgellm.models.layers import PartialSum
    H, S = 4096, 4
    parts = torch.randn(S, M, H, device=cuda)
    res = torch.randn(M, H, device=cuda).bfloat16() if with_res else None
    w = (torch.rand(H, device=cuda) + 0.5).bfloat16()
    y, s, h = ops.rms_norm_parts(parts, res, w, 1e-5, quant)
    x = PartialSum(parts).materialize()
    if quant:
        q_ref, s_ref, h_ref = ops.rms_norm_quant(x, w, 1e-5, res)
        assert torch.equal(y, q_ref) and torch.equal(s, s_ref)
    else:
        y_ref, h_ref = ops.rms_norm(x, w, 1e-5, res)
        assert torch.equal(y, y_ref)
    assert torch.equal(h, h_ref if with_res else x)


def test_model_split_k_decode_matches_unsplit(cuda):
    """W8A8 Llama decode with split-K o/down outputs summed inside the norms == the unsplit path
    (greedy tokens; only float summation order differs)."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    from edgellm.quant import quantize_model
    cfg = tiny("llama2", hidden_size=512, num_heads=4, num_kv_heads=4, intermediate_size=1024, num_layers=2)
    model = quantize_model(build_model(cfg, device=cuda, seed=3), "w8a8_smoothquant")
    lins = [l.attn.o for l in model.layers] + [l.mlp.down for l in model.layers]
    assert all(lin.split_k_out for lin in lins)
    from edgellm.engine import KVCache
    from edgellm.models import AttnCtx
    ids = torch.tensor([[5, 9, 100, 7, 3, 11, 42, 8], [1, 2, 3, 4, 5, 6, 7, 8]] * 2, device=cuda)
    B, T = ids.shape
    logits = {}
    for on in (1, 0):
        for lin in lins:
            lin.split_k_out = on
        kv = KVCache(cfg, B, T + 4, dtype=model.dtype, device=cuda)
        sp = torch.zeros(B, dtype=torch.int32, device=cuda)
        with torch.no_grad():
            last = model(ids, AttnCtx("prefill", B, T, sp, sp + T, T, kv.rows(0, B), model.rope_table(cuda)))
            pos = torch.full((B,), T, dtype=torch.int32, device=cuda)
            logits[on] = model(last.argmax(-1).view(B, 1), AttnCtx("decode", B, 1, pos, pos + 1, T + 1, kv.rows(0, B),
                                                                   model.rope_table(cuda))).float()
    # decode-step logits: only float summation order differs (bounded per row, not token agreement)
    rel = (logits[1] - logits[0]).norm(dim=-1) / logits[0].norm(dim=-1)
    assert rel.max().item() < 2e-2, rel
    sp = SamplingParams(max_new_tokens=12, do_sample=False)
    out = Generator(model, max_batch=4, max_seq=64).generate(ids.tolist(), sp, seed=0).tokens
    assert all(len(t) == 12 for t in out)


@pytest.mark.parametrize("M", [1, 5, 16, 17, 33, 48, 64])
@pytest.mark.parametrize("N,K", [(3072, 2048), (2048, 8192), (7680, 2560), (32000, 4096), (48, 64)])
@pytest.mark.parametrize("bias", [False, True])
def test_gemv_bf16(cuda, M, N, K, bias):
    """bf16 decode GEMV (gemv_bf16.hip) == fp32 reference of x . W^T (+ bias), rounded once."""
    C = ops.ext()
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16() if bias else None
    y = C.gemv_bf16(x, ops.pack_bf16_weight(w), b, N, 0)
    ref = x.float() @ w.float().t() + (b.float() if bias else 0)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    _close(y, ref, 2e-2, 1e-2)
    assert torch.equal(y, C.gemv_bf16(x, ops.pack_bf16_weight(w), b, N, 0))


@pytest.mark.parametrize("M", [1, 7, 16, 31, 64])
@pytest.mark.parametrize("F,K", [(8192, 2048), (5632, 2048), (64, 128)])
def test_gemv_bf16_glu(cuda, M, F, K):
    """Fused bf16 gate_up GEMV + SwiGLU over the natural [gate | up] rows == unfused reference
    (gate and up rounded to bf16, as the GEMM output is)."""
    C = ops.ext()
    torch.manual_seed(F + M)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(2 * F, K, device=cuda) * 0.05).bfloat16()
    h = C.gemv_bf16(x, ops.pack_bf16_weight(w), None, 2 * F, 1)
    gu = (x.float() @ w.float().t()).bfloat16().float()
    g, u = gu[:, :F], gu[:, F:]
    ref = torch.nn.functional.silu(g) * u
    assert h.shape == (M, F)
    _close(h, ref, 2e-2, 2e-2)


def test_linear_bf16_routes_decode_rows(cuda):
    """ops.linear_bf16: <= BF16_GEMV_MAX_ROWS rows take the HIP GEMV, bf16_ring_min_rows..256 the
    bf16 ring GEMM, the rest hipBLASLt; all three agree."""
    torch.manual_seed(0)
    n = ops.BF16_GEMV_MAX_ROWS
    w = (torch.randn(4096, 2048, device=cuda) * 0.05).bfloat16()
    x = torch.randn(300, 2048, device=cuda).bfloat16()
    lo = int(ops.ext().bf16_ring_min_rows())
    assert ops.bf16_decode_mode(x[:n], w) == 1 and ops.bf16_decode_mode(x[:lo], w) == 2
    assert ops.bf16_decode_mode(x[:256], w) == 2 and ops.bf16_decode_mode(x, w) == 0
    assert lo == n + 1 or ops.bf16_decode_mode(x[:n + 1], w) == 0
    small = ops.linear_bf16(x[:n].contiguous(), w)
    ring = ops.linear_bf16(x[:256].contiguous(), w)
    big = ops.linear_bf16(x, w)
    _close(small, big[:n], 2e-2, 1e-2)
    _close(ring, big[:256], 2e-2, 1e-2)


@pytest.mark.parametrize("act", ["gelu_tanh", "gelu"])
@pytest.mark.parametrize("M,N,K", [(1, 10240, 2560), (16, 8192, 2048), (50, 10240, 2560)])
def test_gemv_bf16_gelu(cuda, act, M, N, K):
    """bf16 GEMV with the GELU epilogue == hipBLASLt GEMM -> act_kernel (Phi-2 / Pythia up-proj)."""
    torch.manual_seed(N + M)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    fused = ops.linear_bf16(x, w, b, act=act)
    ref = ops.activation(torch.nn.functional.linear(x, w, b), act)
    _close(fused, ref, 2e-2, 2e-2)


@pytest.mark.parametrize("M", [1, 4, 16])
@pytest.mark.parametrize("K,N", [(2048, 3072), (2560, 10240), (8192, 2048)])
@pytest.mark.parametrize("outliers", [0, 3, 300])
def test_llmint8_device_outliers(cuda, M, K, N, outliers):
    """LLM.int8 decode without a host sync (llmint8.hip, one fused prep kernel) == the uncapped
    any-rows path: the same columns go to the 16-bit part (300 > the decode kernel's 256-column
    cap: the overflow stays int8, so only the first 256 columns may differ from bitsandbytes' split)."""
    from edgellm.models.layers import Linear
    from edgellm.quant import LLMInt8Linear
    torch.manual_seed(M + K + outliers)
    lin = Linear(K, N, bias=True, device=cuda)
    lin.weight.data.copy_(torch.randn(N, K, device=cuda) * 0.02)
    lin.bias.data.copy_(torch.randn(N, device=cuda) * 0.1)
    m = LLMInt8Linear.from_float(lin)
    x = torch.randn(M, K, device=cuda)
    if outliers:
        cols = torch.randperm(K, device=cuda)[:outliers]
        x[0, cols] = 8.0 + torch.rand(outliers, device=cuda) * 4
    x = x.bfloat16()
    fast = m(x)                                         # decode path (M <= 16, one fused prep kernel)
    m_slow = LLMInt8Linear.from_float(lin)
    x_slow = x.float()
    # the uncapped any-rows path (force it with a 17th row of zeros)
    slow = m_slow(torch.cat([x, torch.zeros(17 - M, K, device=cuda, dtype=x.dtype)]))[:M]
    if outliers <= LLMInt8Linear.OUTLIER_CAP:
        _close(fast, slow, 3e-2, 2e-2)
    ref = x_slow @ lin.weight.float().t() + lin.bias.float()
    rel = (fast.float() - ref).norm() / ref.norm()
    assert rel < 2e-2, rel


@pytest.mark.parametrize("K,N", [(2048, 3072), (2560, 10240), (4096, 4096), (2048, 16384), (8192, 2048),
                                 (10240, 2560), (11008, 4096)])
@pytest.mark.parametrize("outliers", [0, 3, 40, 300])
@pytest.mark.parametrize("bias", [True, False])
def test_llmint8_one_launch_exact(cuda, K, N, outliers, bias):
    """Batch-1 LLM.int8 in one launch (gemm_i8.hip l8_prologue: outlier columns, quantisation and the
    outlier part inside the GEMV) == the three-launch decode path (llmint8_prep, the int8 GEMV,
    llmint8_outlier), bit for bit, including past the 256-column cap."""
    from edgellm.models.layers import Linear
    from edgellm.quant import LLMInt8Linear
    torch.manual_seed(K + N + outliers)
    lin = Linear(K, N, bias=bias, device=cuda)
    lin.weight.data.copy_(torch.randn(N, K, device=cuda) * 0.02)
    if bias:
        lin.bias.data.copy_(torch.randn(N, device=cuda) * 0.1)
    m = LLMInt8Linear.from_float(lin)
    x = torch.randn(1, K, device=cuda)
    if outliers:
        x[0, torch.randperm(K, device=cuda)[:outliers]] = 7.0 + torch.rand(outliers, device=cuda) * 4
    x = x.bfloat16()
    one = m(x)                                             # one launch (ONE_LAUNCH)
    m.ONE_LAUNCH = False
    three = m(x)                                           # prep + GEMV + outlier
    assert torch.equal(one, three), (one.float() - three.float()).abs().max()


@pytest.mark.parametrize("K,N", [(2048, 3072), (2560, 10240), (4096, 4096)])
@pytest.mark.parametrize("outliers", [0, 5, 300])
@pytest.mark.parametrize("kind", ["rms", "ln"])
@pytest.mark.parametrize("res", [True, False])
def test_llmint8_norm_one_launch_exact(cuda, K, N, outliers, kind, res):
    """Batch-1 LLM.int8 over RMSNorm / LayerNorm(x + residual) computed in the same launch ==
    the norm kernel followed by the one-launch LLM.int8 projection, bit for bit (output, residual
    row, and the normalised row written for a second consumer)."""
    from edgellm.models.layers import Linear
    from edgellm.quant import LLMInt8Linear
    C = ops.ext()
    torch.manual_seed(K + N + outliers)
    lin = Linear(K, N, bias=True, device=cuda)
    lin.weight.data.copy_(torch.randn(N, K, device=cuda) * 0.02)
    lin.bias.data.copy_(torch.randn(N, device=cuda) * 0.1)
    m = LLMInt8Linear.from_float(lin)
    x = torch.randn(1, K, device=cuda)
    if outliers:
        x[0, torch.randperm(K, device=cuda)[:outliers]] = 30.0
    x = x.bfloat16()
    resid = torch.randn(1, K, device=cuda).bfloat16() if res else None
    gamma = (torch.rand(K, device=cuda) * 2 + 0.5).bfloat16()
    beta = (torch.randn(K, device=cuda) * 0.1).bfloat16() if kind == "ln" else None
    if kind == "rms":
        yr, hr = ops.rms_norm(x, gamma, 1e-5, resid)
    else:
        yr, hr = ops.layer_norm(x, gamma, beta, 1e-5, resid)
    ref = m(yr.contiguous())                               # one launch, over the norm kernel's row
    h, y = torch.empty_like(x), torch.empty_like(x)          # (the call above built m._weight_t)
    out = C.llmint8_gemv_norm(x, resid, gamma, beta, 1e-5, kind == "ln", h, y, m.threshold, m.w_packed,
                              m._w_deq, m.bias, m._weight_t, m.SCB, N, False, 0)
    assert out is not None
    assert torch.equal(h, hr.view_as(h)) and torch.equal(y, yr.view_as(y))
    assert torch.equal(out, ref), (out.float() - ref.float()).abs().max()
    if kind == "rms" and N % 32 == 0:                      # + SwiGLU of [gate | up] in the epilogue
        g = C.llmint8_gemv_norm(x, resid, gamma, beta, 1e-5, False, h, None, m.threshold, m.w_packed,
                                m._w_deq, m.bias, m._weight_t, m.SCB, N, True, 0)
        assert g is not None and g.shape == (1, N // 2)
        assert torch.equal(g, ops.activation(ref, "silu_glu")), (g.float() - ops.activation(ref, "silu_glu").float()).abs().max()
    for act, code in (("gelu_tanh", 1), ("gelu", 2)):                   # + GELU in the epilogue
        g = C.llmint8_gemv_norm(x, resid, gamma, beta, 1e-5, kind == "ln", h, None, m.threshold, m.w_packed,
                                m._w_deq, m.bias, m._weight_t, m.SCB, N, False, code)
        assert g is not None and torch.equal(g, ops.activation(ref, act)), act
        if kind == "rms":                                  # the raw-row form too
            gr = m.gelu_fused(yr.contiguous(), act)
            assert gr is not None and torch.equal(gr, ops.activation(ref, act)), act


@pytest.mark.parametrize("arch", ["llama", "phi", "gpt_neox"])
def test_llmint8_model_norm_fused_matches_unfused(cuda, arch):
    """LLM.int8 Llama / Phi-like / NeoX-like models generate the same greedy tokens at batch 1 with
    the norms inside the one-launch projections as with the norm kernels (gemv_norm 0)."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    from edgellm.quant import quantize_model
    kw = dict(hidden_size=256, num_heads=4, num_kv_heads=4 if arch != "llama" else 2, intermediate_size=1024,
              num_layers=3)
    if arch != "llama":
        kw.update(head_dim=64, rotary_dim=32)
    cfg = tiny(arch, **kw)
    sp = SamplingParams(max_new_tokens=12, do_sample=False)
    C = ops.ext()
    outs = []
    for on in (1, 0):
        C.tune("gemv_norm", on, 0)
        try:
            m = quantize_model(build_model(cfg, device=cuda, seed=13), "llm_int8")
            outs.append(Generator(m, max_batch=1, max_seq=64).generate([[1, 5, 9, 13, 2, 7]], sp, seed=0).tokens)
        finally:
            C.tune("gemv_norm", 1, 0)
    assert outs[0] == outs[1]


def _llmint8_emulation(x, q_w, scb, bias, thr):
    """fp32 emulation of the bitsandbytes split: columns with any |x| > thr in 16-bit against the
    dequantised weight columns, the rest per-token int8 x per-row int8."""
    xf = x.float()
    cols = (xf.abs() > thr).any(0)
    x_in = xf.masked_fill(cols[None, :], 0.0)
    sa = x_in.abs().amax(1).clamp_min(1e-8) / 127.0
    qx = torch.round(x_in / sa[:, None]).clamp(-127, 127)
    w_deq = q_w.float() * (scb.float() / 127.0)[:, None]
    out = (qx @ q_w.float().t()) * sa[:, None] * (scb.float() / 127.0)[None, :]
    out = out + xf[:, cols] @ w_deq[:, cols].t()
    return out + (bias.float() if bias is not None else 0.0), int(cols.sum())


@pytest.mark.parametrize("M", [17, 200, 1000])
@pytest.mark.parametrize("K,N", [(2048, 3072), (4096, 1000)])
@pytest.mark.parametrize("outliers", [0, 5, 300, 1500])
def test_llmint8_rows_device_outliers(cuda, M, K, N, outliers):
    """LLM.int8 at prefill / large-batch rows on the device (llmint8.hip any-rows form, no host
    sync, no column cap) == an fp32 emulation of the bitsandbytes split; every outlier column goes
    to the 16-bit part (1500 columns here, past the decode kernel's 256)."""
    from edgellm.models.layers import Linear
    from edgellm.quant import LLMInt8Linear
    torch.manual_seed(M + K + outliers)
    lin = Linear(K, N, bias=True, device=cuda)
    lin.weight.data.copy_(torch.randn(N, K, device=cuda) * 0.02)
    lin.bias.data.copy_(torch.randn(N, device=cuda) * 0.1)
    m = LLMInt8Linear.from_float(lin)
    x = torch.randn(M, K, device=cuda)
    if outliers:
        cols = torch.randperm(K, device=cuda)[:outliers]
        rows = torch.randint(0, M, (outliers,), device=cuda)      # one row per column: scattered
        x[rows, cols] = (8.0 + torch.rand(outliers, device=cuda) * 4) * torch.sign(torch.randn(outliers, device=cuda))
    x = x.bfloat16()
    C = ops.ext()
    q, sa, cl, count = C.llmint8_prep_rows(x, m.threshold)
    want = torch.nonzero((x.float().abs() > m.threshold).any(0)).flatten()
    assert int(count.item()) == want.numel()
    assert torch.equal(cl[:want.numel()].long(), want)                 # ordered, complete
    out = m(x)
    ref, n_out = _llmint8_emulation(x, m.weight_i8, m.SCB, m.bias, m.threshold)
    assert n_out == want.numel()
    _close(out, ref, 3e-2, 2e-2)
    rel = (out.float() - (x.float() @ lin.weight.float().t() + lin.bias.float())).norm() / ref.norm()
    assert rel < 2e-2, rel


def test_llmint8_rows_graph_capture(cuda):
    """The any-rows LLM.int8 path has static shapes and no host sync: a captured replay equals
    eager on new data with a different outlier set."""
    from edgellm.models.layers import Linear
    from edgellm.quant import LLMInt8Linear
    torch.manual_seed(3)
    K, N, M = 2048, 1024, 96
    lin = Linear(K, N, bias=False, device=cuda)
    lin.weight.data.copy_(torch.randn(N, K, device=cuda) * 0.02)
    m = LLMInt8Linear.from_float(lin)
    assert m.graph_safe_rows >= M
    xin = torch.randn(M, K, device=cuda).bfloat16()
    m(xin)                                              # W^T copy built outside the capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m(xin)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        yout = m(xin)
    x2 = torch.randn(M, K, device=cuda)
    x2[7, torch.randperm(K, device=cuda)[:40]] = 10.0
    xin.copy_(x2.bfloat16())
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(yout, m(xin))


@pytest.mark.parametrize("M", [1, 16, 40, 64])
@pytest.mark.parametrize("N,K,S", [(2048, 8192, 2), (2048, 2048, 2), (4096, 4096, 3)])
def test_gemv_bf16_split_k(cuda, M, N, K, S):
    """bf16 split-K partial slices sum to the unsplit GEMV (fp32 tolerance), bias in slice 0."""
    C = ops.ext()
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    parts = C.gemv_bf16_splitk(x, ops.pack_bf16_weight(w), b, N, S)
    assert parts.shape == (S, M, N) and parts.dtype == torch.float32
    ref = x.float() @ w.float().t() + b.float()
    _close(parts.sum(0), ref, 1e-3, 1e-3)


def test_bf16_model_split_k_decode_matches_unsplit(cuda):
    """A bf16 Llama decodes the same tokens with split-K o/down (PartialSum into the norm) as with
    the plain GEMV."""
    import edgellm.models.decoder as dec
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    cfg = tiny("llama", hidden_size=256, num_heads=4, num_kv_heads=2, intermediate_size=512, num_layers=2)
    sp = SamplingParams(max_new_tokens=8, do_sample=False)
    prompts = [[1, 5, 9, 13, 2, 7], [3, 4, 8, 16, 23, 42]]
    outs = []
    for split in (2, 0):
        m = build_model(cfg, device=cuda, seed=3)
        for layer in m.layers:
            layer.attn.o.split_k_out = layer.mlp.down.split_k_out = split
        outs.append(Generator(m, max_batch=2, max_seq=32).generate(prompts, sp, seed=0).tokens)
    assert outs[0] == outs[1]


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("K,N", [(2048, 3072), (4096, 12288), (2048, 16384), (4096, 22016)])
@pytest.mark.parametrize("S", [1, 2, 3, 4])
@pytest.mark.parametrize("res", [True, False])
@pytest.mark.parametrize("glu", [False, True])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gemv_bf16_norm_prologue_exact(cuda, M, K, N, S, res, glu, dt):
    """16-bit decode GEMV with the RMSNorm in its prologue (gemv_bf16.hip norm16_prologue) ==
    the norm kernel over the split-K slices followed by the plain GEMV: the same output bits and the
    same new residual rows (bf16 and fp16; with / without a residual; plain and SwiGLU epilogues)."""
    torch.manual_seed(M * 7 + K + N + S)
    parts = torch.randn(S, M, K, device=cuda) * 0.5
    resid = torch.randn(M, K, device=cuda).to(dt) if res else None
    gamma = (torch.rand(K, device=cuda) + 0.5).to(dt)
    w = (torch.randn(N, K, device=cuda) * 0.02).to(dt)
    bias = (torch.randn(N, device=cuda) * 0.1).to(dt)
    wp = ops.pack_bf16_weight(w)
    h = torch.empty(M, K, device=cuda, dtype=dt)
    y = ops.gemv_bf16_norm(parts, resid, gamma, 1e-5, h, wp, bias, N, glu=glu)
    wide = (N // 32 if glu else N // 16) >= (512 if glu else 1024)      # the 4-tile geometry
    if K == 4096 and S > 2 and wide:
        assert y is None                                   # not taken (its held slices would spill)
        return
    assert y is not None
    yr, _, hr = ops.rms_norm_parts(parts, resid, gamma, 1e-5, False)
    ref = ops.linear_bf16(yr, w, bias, glu=glu, packed=wp)
    assert torch.equal(h, hr.view_as(h)), "residual rows differ"
    assert torch.equal(y, ref), (y.float() - ref.float()).abs().max()


@pytest.mark.parametrize("M", [1, 3])
@pytest.mark.parametrize("K,N", [(2048, 6144), (2560, 10240), (2560, 2560), (4096, 16384)])
@pytest.mark.parametrize("act", [None, "gelu_tanh", "gelu"])
@pytest.mark.parametrize("res", [True, False])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gemv_bf16_ln_prologue_exact(cuda, M, K, N, act, res, dt):
    """16-bit decode GEMV with the LayerNorm of x (+ residual) in its prologue (gemv_bf16.hip
    ln16_prologue) == the norm kernel followed by the plain / GELU GEMV, bit for bit, and the same
    x + residual rows."""
    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device=cuda).to(dt)
    resid = torch.randn(M, K, device=cuda).to(dt) if res else None
    gamma = (torch.rand(K, device=cuda) + 0.5).to(dt)
    beta = (torch.randn(K, device=cuda) * 0.1).to(dt)
    w = (torch.randn(N, K, device=cuda) * 0.02).to(dt)
    bias = (torch.randn(N, device=cuda) * 0.1).to(dt)
    wp = ops.pack_bf16_weight(w)
    h = torch.empty(M, K, device=cuda, dtype=dt)
    yo = torch.empty(M, K, device=cuda, dtype=dt) if res else None     # the normalised rows too
    y = ops.gemv_bf16_ln(x, resid, gamma, beta, 1e-5, h, wp, bias, N, act, y_out=yo)
    assert y is not None
    yr, hr = ops.layer_norm(x, gamma, beta, 1e-5, resid)
    ref = ops.linear_bf16(yr, w, bias, act=act, packed=wp)
    assert torch.equal(h, hr.view_as(h)), "residual rows differ"
    assert yo is None or torch.equal(yo, yr.view_as(yo)), "normalised rows differ"
    assert torch.equal(y, ref), (y.float() - ref.float()).abs().max()


@pytest.mark.parametrize("arch", ["phi", "gpt_neox"])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_parallel_residual_decode_ln_fused_matches_unfused(cuda, arch, dt):
    """Phi-2-like and GPT-NeoX-like 16-bit models generate the same greedy tokens at batch 1 with
    their LayerNorms in the qkv / up GEMV prologues as with the norm kernels (gemv_norm 0)."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    cfg = tiny(arch, hidden_size=256, num_heads=4, num_kv_heads=4, head_dim=64, intermediate_size=1024,
               rotary_dim=32, num_layers=3)
    sp = SamplingParams(max_new_tokens=12, do_sample=False)
    C = ops.ext()
    outs = []
    for on in (1, 0):
        C.tune("gemv_norm", on, 0)
        try:
            m = build_model(cfg, dtype=dt, device=cuda, seed=11)
            outs.append(Generator(m, max_batch=1, max_seq=64).generate([[1, 5, 9, 13, 2, 7]], sp, seed=0).tokens)
        finally:
            C.tune("gemv_norm", 1, 0)
    assert outs[0] == outs[1]


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("K,N", [(2048, 6144), (2048, 8192), (2560, 10240), (4096, 4096)])
@pytest.mark.parametrize("geluq", [None, "gelu_tanh", "gelu"])
@pytest.mark.parametrize("res", [True, False])
def test_w8a8_gemv_ln_prologue_exact(cuda, M, K, N, geluq, res):
    """W8A8 decode GEMV with LayerNorm + per-token int8 of bf16 rows in its prologue (gemm_i8.hip
    ln_prologue) == layer_norm_quant followed by the plain / quantising-GELU GEMV, bit for bit."""
    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device=cuda).bfloat16()
    resid = torch.randn(M, K, device=cuda).bfloat16() if res else None
    gamma = (torch.rand(K, device=cuda) + 0.5).bfloat16()
    beta = (torch.randn(K, device=cuda) * 0.1).bfloat16()
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = (torch.randn(N, device=cuda) * 0.1).bfloat16()
    wp = ops.pack_int8_weight(w)
    h = torch.empty(M, K, device=cuda, dtype=torch.bfloat16)
    r = ops.w8a8_gemv_ln(x, resid, gamma, beta, 1e-5, h, wp, sw, bias, N, K, geluq=geluq)
    assert r is not None
    q, s, hr = ops.layer_norm_quant(x, gamma, beta, 1e-5, resid)
    assert torch.equal(h, hr.view_as(h)), "residual rows differ"
    if geluq is None:
        ref = ops.w8a8_linear(q, s, wp, sw, bias, N, K)
        assert torch.equal(r, ref), (r.float() - ref.float()).abs().max()
    else:
        qr, sr = ops.w8a8_geluq(q, s, wp, sw, bias, N, K, geluq)
        assert torch.equal(r[0], qr)
        assert torch.equal(r[1][:, :M], sr[:, :M])


def test_neox_w8a8_decode_ln_fused_matches_unfused(cuda):
    """A GPT-NeoX-like W8A8 model generates the same greedy tokens at batch 1 with its two
    LayerNorms (+ int8 quant) in the qkv / up GEMV prologues as with the norm kernels."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    from edgellm.quant import quantize_model
    cfg = tiny("gpt_neox", hidden_size=256, num_heads=4, num_kv_heads=4, head_dim=64, intermediate_size=1024,
               rotary_dim=32, num_layers=3)
    sp = SamplingParams(max_new_tokens=12, do_sample=False)
    C = ops.ext()
    outs = []
    for on in (1, 0):
        C.tune("gemv_norm", on, 0)
        try:
            m = quantize_model(build_model(cfg, device=cuda, seed=11), "w8a8_smoothquant")
            outs.append(Generator(m, max_batch=1, max_seq=64).generate([[1, 5, 9, 13, 2, 7]], sp, seed=0).tokens)
        finally:
            C.tune("gemv_norm", 1, 0)
    assert outs[0] == outs[1]


def test_bf16_llama_decode_norm_fused_matches_unfused(cuda):
    """A bf16 Llama (hidden 2048: the prologue's K) generates the same greedy tokens at batch 1
    with its RMSNorms in the qkv / gate_up GEMV prologues as with the norm kernels (gemv_norm 0),
    and the fused step has two launches fewer per layer."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    cfg = tiny("llama", hidden_size=2048, num_heads=16, num_kv_heads=4, intermediate_size=4096, num_layers=2)
    sp = SamplingParams(max_new_tokens=12, do_sample=False)
    C = ops.ext()
    outs = []
    for on in (1, 0):
        C.tune("gemv_norm", on, 0)
        try:
            m = build_model(cfg, device=cuda, seed=5)
            outs.append(Generator(m, max_batch=1, max_seq=64).generate([[1, 5, 9, 13, 2, 7]], sp, seed=0).tokens)
        finally:
            C.tune("gemv_norm", 1, 0)
    assert outs[0] == outs[1]


@pytest.mark.parametrize("M", [65, 100, 128])
@pytest.mark.parametrize("N,K,S", [(12288, 4096, 1), (6144, 4096, 1), (12304, 4096, 1), (4096, 4096, 4),
                                   (4096, 11008, 4)])
def test_ring2_rows128_exact(cuda, M, N, K, S):
    """65-128 rows on the ring2 kernel with per-token scales: the int32 sums are exact, so whole-K
    outputs equal the prefill GEMM's (same epilogue arithmetic) and split-K slices are
    deterministic and sum to the fp32 reference."""
    C = ops.ext()
    torch.manual_seed(M + N)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    if S == 1:
        out = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        try:
            C.tune("gemv_ring", 0, 0)                # no decode ring: the prefill GEMM takes 65+ rows
            big = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        finally:
            C.tune("gemv_ring", 2, 0)
        _close(out, ref, 1e-2, 1e-2)
        _close(out, big, 0, 1e-2)                    # bf16 rounding of the same fp32 value at most
        return
    parts = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, S)
    assert torch.equal(parts, C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, S))
    _close(parts.sum(0), ref, 1e-3, 1e-2)


@pytest.mark.parametrize("M", [65, 100, 128])
@pytest.mark.parametrize("N,K,S", [(4096, 4096, 4), (4096, 11008, 4), (1024, 14336, 4)])
def test_ring2_grouped_splitk(cuda, M, N, K, S):
    """o / down at 65-128 rows: the decoupled-depth ring kernel with per-(token, 64) scales folded
    per k-tile and split-K slices on stage boundaries: deterministic, and the slice sums match the
    fp32 reference."""
    C = ops.ext()
    torch.manual_seed(M * 7 + K)
    Mpad = (M + 15) // 16 * 16
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(K // 64, Mpad, device=cuda) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    p2 = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, S)
    again = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, S)
    assert torch.equal(p2, again)                      # deterministic
    s2 = p2.sum(0)
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    _close(s2, ref, 1e-3, 1e-2)


@pytest.mark.parametrize("act", ["gelu_tanh", "gelu"])
@pytest.mark.parametrize("M", [1, 5, 16, 33, 64])
@pytest.mark.parametrize("N,K", [(10240, 2560), (8192, 2048), (128, 192)])
def test_w8a8_geluq_matches_reference(cuda, act, M, N, K):
    """Fused up projection + GELU + per-(token, 64) int8 (the GELU MLPs' decode path) == the
    reference composition w8a8_linear -> bf16 -> gelu -> quant_per_group (dequantised values within
    one int8 step of the group scale; scales to 1e-3 relative)."""
    torch.manual_seed(M + N + (act == "gelu"))
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.004 + 1e-4
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.004 + 1e-4
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    q, s = ops.w8a8_geluq(qx, sx, wp, sw, bias, N, K, act)
    Mpad = (M + 15) // 16 * 16
    assert q.shape == (M, N) and s.shape == (N // 64, Mpad)
    assert (s[:, M:] == 0).all()
    y = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.bfloat16)
    rq, rs = _ref.quant_per_group(_ref.gelu(y, "tanh" if act == "gelu_tanh" else "none"))
    _close(s[:, :M], rs[:, :M], 0.0, 1e-3)
    step = s[:, :M].t().repeat_interleave(64, dim=1)
    deq, rdeq = q.float() * step, rq.float() * rs[:, :M].t().repeat_interleave(64, dim=1)
    assert ((deq - rdeq).abs() <= step * 1.01 + 1e-6).all()


def test_w8a8_gelu_mlp_takes_fused_path(cuda):
    """A W8A8 Phi-style (GELU, parallel residual) decoder at decode rows routes its MLP through the
    fused GELU-quant kernel and stays close to the bf16 model at the logits."""
    from edgellm.engine import KVCache
    from edgellm.models import AttnCtx, build_model, tiny
    from edgellm.quant import quantize_model
    cfg = tiny("phi", hidden_size=256, num_heads=4, num_kv_heads=4, intermediate_size=1024, num_layers=2)
    base = build_model(cfg, device=cuda, seed=3)
    qm = quantize_model(build_model(cfg, device=cuda, seed=3), "w8a8")
    B, T = 4, 12
    ids = torch.randint(0, cfg.vocab_size, (B, T), generator=torch.Generator().manual_seed(0)).to(cuda)
    outs = []
    for m in (base, qm):
        kv = KVCache(cfg, B, T + 4, dtype=m.dtype, device=cuda)
        sp = torch.zeros(B, dtype=torch.int32, device=cuda)
        with torch.no_grad():
            m(ids, AttnCtx("prefill", B, T, sp, sp + T, T, kv.rows(0, B), m.rope_table(cuda)), logits="last")
            pos = torch.full((B,), T, dtype=torch.int32, device=cuda)
            outs.append(m(ids[:, -1:], AttnCtx("decode", B, 1, pos, pos + 1, T + 1, kv.rows(0, B),
                                               m.rope_table(cuda))).float())
    mlp = qm.layers[0].mlp
    assert getattr(mlp.up, "geluq_rows_ok", lambda m: False)(B)
    rel = ((outs[1] - outs[0]).norm() / outs[0].norm()).item()
    assert rel < 0.1, rel


@pytest.mark.parametrize("M", [1, 16, 40])
def test_gemv_addend_matches_unfused_add(cuda, M):
    """Parallel-residual fusion: the W8A8 (grouped and per-token scales) and bf16 decode GEMVs add a
    bf16 addend in their epilogue == bf16(bf16(y) + addend), the unfused add, bit for bit."""
    torch.manual_seed(M)
    N, K = 2560, 10240
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.004 + 1e-4
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    add = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    C = ops.ext()
    Mpad = (M + 15) // 16 * 16
    for sx in (torch.rand(M, device=cuda) * 0.004 + 1e-4, torch.rand(K // 64, Mpad, device=cuda) * 0.004 + 1e-4):
        y = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        fused = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K, add)
        assert torch.equal(fused, y + add)
    xb = torch.randn(M, K, device=cuda).bfloat16()
    wb = (torch.randn(N, K, device=cuda) * 0.02).bfloat16()
    wpb = ops.pack_bf16_weight(wb)
    yb = C.gemv_bf16(xb, wpb, bias, N, 0)
    assert torch.equal(C.gemv_bf16(xb, wpb, bias, N, 0, add), yb + add)


@pytest.mark.parametrize("M", [1, 3, 4])
@pytest.mark.parametrize("K,S", [(4096, 2), (4096, 1), (4096, 4), (2048, 4), (2048, 3)])
def test_gemv_norm_prologue_bit_exact(cuda, K, S, M):
    """Decode RMSNorm (1-4 rows) in the consuming W8A8 GEMV's prologue (ops.w8a8_gemv_norm) == the
    norm kernel over the split-K slices (ops.rms_norm_parts) followed by the plain GEMV / quantising
    SwiGLU GEMV, bit for bit, and the new residual rows it writes == the norm kernel's."""
    torch.manual_seed(K + S + M)
    parts = torch.randn(S, M, K, device=cuda) * 0.5
    res = torch.randn(M, K, device=cuda).bfloat16()
    gamma = (torch.rand(K, device=cuda) + 0.5).bfloat16()
    eps = 1e-5
    q, s, r = ops.rms_norm_parts(parts, res, gamma, eps, True)
    for N, glu in ((3 * K, False), (2 * 4 * K, True), (4 * K + 48, False)):
        w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
        wp = ops.pack_int8_weight(w)
        sw = torch.rand(N, device=cuda) * 0.004 + 1e-4
        bias = torch.randn(N, device=cuda).bfloat16()
        h = torch.full((M, K), float("nan"), device=cuda).bfloat16()
        fused = ops.w8a8_gemv_norm(parts, res, gamma, eps, h, wp, sw, bias, N, K, glu_quant=glu)
        assert fused is not None
        assert torch.equal(h, r)
        if glu:
            ref = ops.w8a8_glu(q, s, wp, sw, bias, N, K, quant=True)
            assert torch.equal(fused[0], ref[0]) and torch.equal(fused[1], ref[1])
        else:
            assert torch.equal(fused, ops.w8a8_linear(q, s, wp, sw, bias, N, K))


def test_gemv_norm_declines_unsupported(cuda):
    """Shapes outside the prologue's layout return None (the caller runs the norm kernel)."""
    K, N = 4096, 4096
    wp = ops.pack_int8_weight(torch.zeros(N, K, dtype=torch.int8, device=cuda))
    sw = torch.ones(N, device=cuda)
    res = torch.zeros(1, K, device=cuda).bfloat16()
    g = torch.ones(K, device=cuda).bfloat16()
    h = torch.empty(1, K, device=cuda).bfloat16()
    assert not ops.gemv_norm_ok(torch.zeros(5, 1, K, device=cuda))
    assert not ops.gemv_norm_ok(torch.zeros(2, 5, K, device=cuda))
    assert ops.gemv_norm_ok(torch.zeros(2, 1, K, device=cuda))
    assert ops.gemv_norm_ok(torch.zeros(2, 4, K, device=cuda)) == (ops.NORM_FUSE_MAX_ROWS >= 4)
    assert ops.w8a8_gemv_norm(torch.zeros(5, 1, K, device=cuda), res, g, 1e-5, h, wp, sw, None, N, K) is None


@pytest.mark.parametrize("B", [1, 4])
def test_llama_batch1_decode_defers_norms(cuda, B, monkeypatch):
    """A W8A8 Llama decoder (hidden 2048) at 1-4 rows runs its inner RMSNorms in the qkv / gate_up
    GEMV prologues and produces the same logits as with the norm kernels (knob gemv_norm=0)."""
    from edgellm.engine import KVCache
    from edgellm.models import AttnCtx, build_model, tiny
    from edgellm.models.layers import PendingNorm
    from edgellm.quant import quantize_model
    cfg = tiny("llama", hidden_size=2048, num_heads=16, num_kv_heads=4, intermediate_size=4096, num_layers=3)
    qm = quantize_model(build_model(cfg, device=cuda, seed=5), "w8a8")
    T = 9
    ids = torch.randint(0, cfg.vocab_size, (B, T), generator=torch.Generator().manual_seed(1)).to(cuda)
    seen = []
    orig = qm.layers[1].attn.qkv.forward

    def spy(x, add=None):
        seen.append(isinstance(x, PendingNorm))
        return orig(x, add)

    qm.layers[1].attn.qkv.forward = spy
    monkeypatch.setattr(ops, "NORM_FUSE_MAX_ROWS", 4)      # the default fuses at batch 1 only
    C = ops.ext()
    outs = []
    try:
        for on in (1, 0):
            C.tune("gemv_norm", on, 0)
            kv = KVCache(cfg, B, T + 4, dtype=qm.dtype, device=cuda)
            sp = torch.zeros(B, dtype=torch.int32, device=cuda)
            with torch.no_grad():
                qm(ids, AttnCtx("prefill", B, T, sp, sp + T, T, kv.rows(0, B), qm.rope_table(cuda)), logits="last")
                pos = torch.full((B,), T, dtype=torch.int32, device=cuda)
                outs.append(qm(ids[:, -1:], AttnCtx("decode", B, 1, pos, pos + 1, T + 1, kv.rows(0, B),
                                                    qm.rope_table(cuda))).float())
    finally:
        C.tune("gemv_norm", 1, 0)
        del qm.layers[1].attn.qkv.forward
    assert seen == [False, True, False, False], seen        # prefill, decode (knob on), prefill, decode
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B", [1, 4])
def test_first_norm_deferred_over_fp32_embedding(cuda, B, monkeypatch):
    """At batch 1 (<= NORM_FUSE_MAX_ROWS rows) the first layer's RMSNorm runs in its qkv GEMV's
    prologue over the embedding handed over as one fp32 slice with no residual
    (DecoderLM.embed_tokens -> PartialSum): decode logits and the residual stream equal the
    bf16-embedding path's bit for bit."""
    from edgellm.engine import KVCache
    from edgellm.models import AttnCtx, build_model, tiny
    from edgellm.models.decoder import DecoderLM
    from edgellm.quant import quantize_model
    cfg = tiny("llama", hidden_size=2048, num_heads=16, num_kv_heads=4, intermediate_size=4096, num_layers=2)
    qm = quantize_model(build_model(cfg, device=cuda, seed=6), "w8a8")
    monkeypatch.setattr(ops, "NORM_FUSE_MAX_ROWS", 4)
    T = 7
    ids = torch.randint(0, cfg.vocab_size, (B, T), generator=torch.Generator().manual_seed(3)).to(cuda)
    assert qm._first_norm_deferred(B)
    outs = []
    for on in (True, False):
        if not on:
            monkeypatch.setattr(DecoderLM, "_first_norm_deferred", lambda self, rows: False)
        kv = KVCache(cfg, B, T + 4, dtype=qm.dtype, device=cuda)
        sp = torch.zeros(B, dtype=torch.int32, device=cuda)
        with torch.no_grad():
            qm(ids, AttnCtx("prefill", B, T, sp, sp + T, T, kv.rows(0, B), qm.rope_table(cuda)), logits="last")
            pos = torch.full((B,), T, dtype=torch.int32, device=cuda)
            outs.append(qm(ids[:, -1:], AttnCtx("decode", B, 1, pos, pos + 1, T + 1, kv.rows(0, B),
                                                qm.rope_table(cuda))).float())
    assert torch.equal(outs[0], outs[1])

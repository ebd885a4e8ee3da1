"""129-256-row decode GEMMs (gemm_i8.hip ``launch_rows256``: ring2 with the rows split in two
halves that stream one weight panel on the same XCD) against the fp32 reference ops.

One 256-row decode micro-batch reads every weight from HBM once per step, where two 128-row
lanes read it twice.  Every geometry the launcher picks is covered: whole-K bf16 outputs (qkv), split-K fp32 partial slices
with per-(token, 64) or per-token activation scales (o / down), and the quantising SwiGLU
epilogue (gate_up).
"""
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


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("N,K", [(12288, 4096), (6144, 4096), (4096, 4096), (2560, 2560), (22016, 4096)])
def test_rows256_out(cuda, M, N, K):
    C = ops.ext()
    assert C.rows256_ok(K)
    torch.manual_seed(M + N + K)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    out = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
    again = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
    assert torch.equal(out, again)
    _close(out, ref, 1e-2, 1e-2)


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("grouped", [True, False])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (1024, 14336)])
def test_rows256_splitk(cuda, M, grouped, N, K):
    """Split-K slices vs the fp32 reference.  Grouped scales: the one-VALU magic-number fold
    (gemm_i8.hip DT = 2) rounds within 8 biased terms per accumulator, so it is held to 1e-4 of
    the output's largest magnitude (measured 4.2-4.7e-5); per-token scales (exact int32 sums) to
    the exact-integer tolerance."""
    C = ops.ext()
    torch.manual_seed(M * 7 + K)
    Mpad = (M + 15) // 16 * 16
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = (torch.rand(K // 64, Mpad, device=cuda) if grouped else torch.rand(M, device=cuda)) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    parts = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, 0)
    again = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, 0)
    S = 4 if K // 128 >= 64 else 2
    assert parts.shape == (S, M, N)
    assert torch.equal(parts, again)
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    atol = max(1e-3, 1e-4 * ref.abs().max().item()) if grouped else 1e-3
    _close(parts.sum(0), ref, atol, 1e-2)


@pytest.mark.parametrize("M", [129, 256])
@pytest.mark.parametrize("F,K", [(11008, 4096), (14336, 4096), (1024, 2048), (1088, 2048)])
def test_rows256_gluq(cuda, M, F, K):
    C = ops.ext()
    torch.manual_seed(M + F)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.004 + 1e-4
    w = torch.randint(-127, 128, (2 * F, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(2 * F, device=cuda) * 0.004 + 1e-4
    bias = torch.randn(2 * F, device=cuda).to(torch.bfloat16)
    wb, swb, bb = _ref.block_glu_rows(w), _ref.block_glu_rows(sw), _ref.block_glu_rows(bias)
    wp = ops.pack_int8_weight(wb)
    ref = _ref.silu_mul(_ref.unblock_glu(_ref.w8a8_linear(qx, sx, wb, swb, bb, torch.bfloat16)))
    q, s = C.w8a8_gemm_gluq(qx, sx, wp, swb, bb, 2 * F, K)
    Mpad = (M + 15) // 16 * 16
    assert s.shape == (F // 64, Mpad)
    assert (s[:, M:] == 0).all()
    step = s[:, :M].t().unsqueeze(-1)
    deq = q.float().view(M, F // 64, 64) * step
    err = (deq - ref.float().view(M, F // 64, 64)).abs()
    assert (err <= 0.51 * step + 1e-2 * ref.float().view(M, F // 64, 64).abs() + 1e-3).all(), err.max().item()


def test_rows256_model_routes(cuda):
    """A W8A8 Llama layer stack at 256 decode rows takes the fused path: grouped-scale attention
    output, split-K o / down partials, quantising GLU (decode_rows_ok routes 129-256 rows)."""
    assert ops.decode_rows_ok(256, 4096) and ops.decode_rows_ok(256, 11008, 4)
    assert not ops.decode_rows_ok(257, 4096)


def _r256(C, on):
    class _Ctx:
        def __enter__(self):
            C.tune("r256_packed", on, 0)

        def __exit__(self, *a):
            C.tune("r256_packed", 1, 0)
            return False
    return _Ctx()


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("H", [4096, 2048])
@pytest.mark.parametrize("parts", [0, 2])
def test_norm_packed_output_is_pack_of_rows(cuda, M, H, parts):
    """The norm kernel's fragment-packed int8 output (quant = 2) is exactly pack_a of its row-major
    output (same values and scales), and ops.unpack_a inverts it."""
    C = ops.ext()
    torch.manual_seed(M + H + parts)
    w = (torch.rand(H, device=cuda) + 0.5).to(torch.bfloat16)
    res = torch.randn(M, H, device=cuda).to(torch.bfloat16)
    if parts:
        xp = torch.randn(parts, M, H, device=cuda)
        q0, s0, r0 = C.rms_norm_parts(xp, res, w, 1e-5, 1)
        q1, s1, r1 = C.rms_norm_parts(xp, res, w, 1e-5, 2)
    else:
        x = torch.randn(M, H, device=cuda).to(torch.bfloat16)
        q0, s0, r0 = C.norm(x, res, w, None, 1e-5, True, 1)
        q1, s1, r1 = C.norm(x, res, w, None, 1e-5, True, 2)
    assert torch.equal(s0, s1) and torch.equal(r0, r1)
    assert q1.shape == (M, H) and q1.stride(0) == H
    assert torch.equal(ops.unpack_a(q1, M, H), q0)


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("N,K", [(12288, 4096), (6144, 4096), (4096, 4096), (6144, 2048), (2048, 2048)])
def test_r256_packed_equals_ring2(cuda, M, N, K):
    """The packed-activation 256-row kernel (w8a8_r256_kernel: activations global -> VGPR, only
    the weight panel through LDS) is bit-identical to the row-major ring2 kernel, and within the
    fp32 reference's tolerance."""
    C = ops.ext()
    assert ops.r256_ok(M, N, K)
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w_n = (torch.rand(K, device=cuda) + 0.5).to(torch.bfloat16)
    qx, sx, _ = C.norm(x, None, w_n, None, 1e-5, True, 1)
    qp, sp, _ = C.norm(x, None, w_n, None, 1e-5, True, 2)
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    ring = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
    out = ops.w8a8_r256(qp, sp, wp, sw, bias, N, K)
    assert out is not None and torch.equal(out, ring)
    _close(out, _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32), 1e-2, 1e-2)


def test_r256_model_logits_unchanged(cuda):
    """A W8A8 Llama decoder at 256 decode rows: the packed qkv path (norm1 writes packed rows, qkv
    runs w8a8_r256) gives bit-identical logits to the row-major ring2 path."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    from edgellm.quant import quantize_model
    C = ops.ext()
    cfg = tiny("llama2", num_layers=2, hidden_size=2048, intermediate_size=5504, num_heads=16, num_kv_heads=16,
               head_dim=128, vocab_size=1024)
    model = quantize_model(build_model(cfg, device=cuda, seed=3), "w8a8_smoothquant")
    prompts = torch.randint(0, cfg.vocab_size, (256, 9), generator=torch.Generator().manual_seed(1)).tolist()
    sp = SamplingParams(max_new_tokens=6, do_sample=False, repetition_penalty=1.1)
    outs = []
    for on in (1, 0):
        with _r256(C, on):
            gen = Generator(model, max_batch=256, max_seq=32, use_graphs=False)
            outs.append(gen.generate(prompts, sp).tokens)
    assert outs[0] == outs[1]


def _wreg(C, da):
    class _Ctx:
        def __enter__(self):
            C.tune("r256_wreg", da, 0)

        def __exit__(self, *a):
            C.tune("r256_wreg", 0, 0)
            return False
    return _Ctx()


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("N", [12288, 4096, 22016, 2560])
@pytest.mark.parametrize("da", [4, 6])
def test_wreg_out_equals_ring2(cuda, M, N, da):
    """The weights-in-VGPR 256-row kernel (gemm_i8_wreg.hip, EPI_OUT) gives ring2's bf16 outputs
    bit for bit (the same exact int32 sums and fp32 epilogue) and matches the fp32 reference."""
    C = ops.ext()
    K = 4096
    torch.manual_seed(M + N + da)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    want = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
    with _wreg(C, da):
        got = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        again = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
    torch.cuda.synchronize()
    assert torch.equal(got, again)
    _close(got, _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32), 1e-2, 1e-2)
    assert torch.equal(got, want)


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("F", [11008, 14336, 1024, 1152])
def test_wreg_gluq_equals_ring2(cuda, M, F):
    """The weights-in-VGPR quantising gate_up (SwiGLU + int8 per (token, 64 features), the amax
    completed across 4 waves through LDS) gives ring2's int8 rows and scales exactly."""
    C = ops.ext()
    K = 4096
    torch.manual_seed(M + F)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.004 + 1e-4
    w = torch.randint(-127, 128, (2 * F, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(2 * F, device=cuda) * 0.004 + 1e-4
    bias = torch.randn(2 * F, device=cuda).to(torch.bfloat16)
    wb, swb, bb = _ref.block_glu_rows(w), _ref.block_glu_rows(sw), _ref.block_glu_rows(bias)
    wp = ops.pack_int8_weight(wb)
    q0, s0 = C.w8a8_gemm_gluq(qx, sx, wp, swb, bb, 2 * F, K)
    with _wreg(C, 4):
        q1, s1 = C.w8a8_gemm_gluq(qx, sx, wp, swb, bb, 2 * F, K)
    torch.cuda.synchronize()
    assert torch.equal(s1, s0)
    assert torch.equal(q1, q0)

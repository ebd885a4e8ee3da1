"""129-256-row decode GEMMs (gemm_i8.hip ``launch_rows256``: ring2 with the rows split in two
halves that stream one weight panel on the same XCD) against the fp32 reference ops.

One 256-row decode micro-batch reads every weight from HBM once per step, where two 128-row
lanes read it twice.  Every geometry the launcher picks and the per-workgroup k rotation
(``tune("ring2_256_rot", 1)``) are covered: whole-K bf16 outputs (qkv), split-K fp32 partial slices
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


def _tuned(C, rot):
    class _Ctx:
        def __enter__(self):
            C.tune("ring2_256_rot", rot, 0)

        def __exit__(self, *a):
            C.tune("ring2_256_rot", 0, 0)
            return False
    return _Ctx()


@pytest.mark.parametrize("rot", [0, 1])
@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("N,K", [(12288, 4096), (6144, 4096), (4096, 4096), (2560, 2560), (22016, 4096)])
def test_rows256_out(cuda, rot, M, N, K):
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
    with _tuned(C, rot):
        out = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        again = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
    assert torch.equal(out, again)
    _close(out, ref, 1e-2, 1e-2)


@pytest.mark.parametrize("rot", [0, 1])
@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("grouped", [True, False])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (1024, 14336)])
def test_rows256_splitk(cuda, rot, M, grouped, N, K):
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
    with _tuned(C, rot):
        parts = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, 0)
        again = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, 0)
    S = 4 if K // 128 >= 64 else 2
    assert parts.shape == (S, M, N)
    assert torch.equal(parts, again)
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    atol = max(1e-3, 1e-4 * ref.abs().max().item()) if grouped else 1e-3
    _close(parts.sum(0), ref, atol, 1e-2)


@pytest.mark.parametrize("rot", [0, 1])
@pytest.mark.parametrize("M", [129, 256])
@pytest.mark.parametrize("F,K", [(11008, 4096), (14336, 4096), (1024, 2048), (1088, 2048)])
def test_rows256_gluq(cuda, rot, M, F, K):
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
    with _tuned(C, rot):
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

"""Prefill INT8 GEMM on v_mfma_i32_32x32x32_i8 (gemm_i8.hip ``w8a8_gemm_x32_kernel``, 256 x 256
block tiles, staggered DMA issue) against the 16x16x64 kernel (bit-equal) and the fp32 reference op,
row-major and fragment-packed A (the APK path at >= 2048 rows x N >= 8192), ragged M.  tune
"prefill_x32" 2 takes it from 192 tiles so the small shapes run it too; 1 (default) from 512."""
import pytest
import torch

from edgellm import ops
from edgellm.ops import _ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [256, 777, 2048, 4100])
@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 11008), (22016, 4096)])
def test_prefill_x32_matches_reference(cuda, M, N, K):
    C = ops.ext()
    torch.manual_seed(M + N)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    try:
        C.tune("prefill_x32", 0, 0)
        base = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        C.tune("prefill_x32", 2, 0)
        out = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
    finally:
        C.tune("prefill_x32", 1, 0)
    # int32 sums are exact in any order: the same bits as the 16x16x64 kernel
    assert torch.equal(out, base)
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    err = (out.float() - ref).abs()
    assert (err <= 1e-2 + 1e-2 * ref.abs()).all(), err.max().item()


@pytest.mark.parametrize("M,N,K", [(1000, 22016, 4096), (2048, 22016, 4096), (2048, 6144, 1024)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_prefill_gate_up_swiglu_epilogue(cuda, M, N, K, with_bias):
    """gate_up (16-blocked [gate | up] columns) with silu(g) * u in the x32 kernel's epilogue ==
    the GEMM's bf16 output through the blocked activation kernel, bit for bit (g and u are rounded to
    bf16 first, as the unfused path stores them), with and without the fragment-packed A copy."""
    C = ops.ext()
    torch.manual_seed(M + N)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16) if with_bias else None
    wp = ops.pack_int8_weight(w)
    try:
        C.tune("prefill_x32", 2, 0)                  # the x32 kernel from 192 tiles (small test grids)
        g_u = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        h = C.w8a8_prefill_glu(qx, sx, wp, sw, bias, N, K)
        C.tune("prefill_apack", 2, 0)
        h_pk = C.w8a8_prefill_glu(qx, sx, wp, sw, bias, N, K)
    finally:
        C.tune("prefill_x32", 1, 0)
        C.tune("prefill_apack", 1, 0)
    assert h is not None and h.shape == (M, N // 2)
    ref = ops.activation(g_u, "silu_glu_blocked")
    assert torch.equal(h, ref)
    assert torch.equal(h_pk, ref)


def test_prefill_gate_up_swiglu_declines_small_grids(cuda):
    """Below the x32 kernel's grid threshold the fused op returns None (the caller keeps the GEMM +
    activation kernel path)."""
    C = ops.ext()
    qx = torch.randint(-127, 128, (100, 1024), dtype=torch.int8, device=cuda)
    sx = torch.rand(100, device=cuda)
    wp = ops.pack_int8_weight(torch.randint(-127, 128, (512, 1024), dtype=torch.int8, device=cuda))
    sw = torch.rand(512, device=cuda)
    assert C.w8a8_prefill_glu(qx, sx, wp, sw, None, 512, 1024) is None

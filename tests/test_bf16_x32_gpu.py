"""bf16 prefill GEMM on v_mfma_f32_32x32x16_bf16 (gemm_i8.hip ``w8a8_gemm_x32_kernel`` DT = 1, 256 x 256
tiles over the fragment-packed bf16 weight) against the fp32 reference and hipBLASLt."""
import pytest
import torch

from edgellm import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [256, 1000, 4096])
@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 11008), (22016, 4096), (2048, 2048)])
def test_bf16_x32_matches_reference(cuda, M, N, K):
    C = ops.ext()
    torch.manual_seed(M + N + K)
    x = (torch.randn(M, K, device=cuda) * 0.5).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.02).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    y = C.gemm_bf16_x32(x, ops.pack_bf16_weight(w), b, N)
    if y is None:                                   # too few tiles for the kernel: hipBLASLt's shape
        assert (M + 255) // 256 * ((N + 255) // 256) < 192
        return
    ref = x.float() @ w.float().t() + b.float()
    err = (y.float() - ref).abs()
    assert (err <= 2e-2 + 1e-2 * ref.abs()).all(), err.max().item()
    blas = torch.nn.functional.linear(x, w, b).float()
    assert (y.float() - blas).abs().max().item() <= 4e-2 + 1e-2 * blas.abs().max().item()

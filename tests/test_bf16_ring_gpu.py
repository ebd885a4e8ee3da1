"""bf16 decode GEMM at 17-256 rows (gemm_i8.hip ring2 kernel in bf16 operand mode) against the
fp32 reference of the same op: plain output (+ bias), the fused SwiGLU over natural [gate | up]
rows, and split-K fp32 partial slices; 129-256 rows run as two row halves (MS = 2).  Model level:
tests/test_decode_numerics_gpu.py (bf16 Llama-2-7B layers at 64 / 128 / 200 / 256 decode rows)."""
import pytest
import torch

from edgellm import ops

pytestmark = pytest.mark.gpu

ROWS = [17, 32, 64, 100, 128, 129, 200, 256]


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    bad = (err > atol + rtol * b.abs()).sum().item()
    assert bad == 0, f"{bad} / {a.numel()} elements off, max err {err.max().item():.4g}"


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 4096), (32000, 4096), (3072, 2048), (48, 128)])
def test_ring_bf16_out(cuda, M, N, K):
    C = ops.ext()
    torch.manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16() if N % 3 == 0 else None
    y = C.gemm_bf16_ring(x, ops.pack_bf16_weight(w), b, N, 0, 0)
    ref = x.float() @ w.float().t() + (b.float() if b is not None else 0)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    _close(y, ref, 2e-2, 1e-2)
    assert torch.equal(y, C.gemm_bf16_ring(x, ops.pack_bf16_weight(w), b, N, 0, 0))   # deterministic


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("F,K", [(11008, 4096), (8192, 2048), (64, 128)])
def test_ring_bf16_glu(cuda, M, F, K):
    C = ops.ext()
    torch.manual_seed(F + M)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(2 * F, K, device=cuda) * 0.05).bfloat16()
    h = C.gemm_bf16_ring(x, ops.pack_bf16_weight(w), None, 2 * F, 1, 0)
    gu = (x.float() @ w.float().t()).bfloat16().float()
    g, u = gu[:, :F], gu[:, F:]
    ref = torch.nn.functional.silu(g) * u
    assert h.shape == (M, F)
    _close(h, ref, 2e-2, 2e-2)


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (2048, 8192)])
def test_ring_bf16_splitk(cuda, M, N, K):
    C = ops.ext()
    torch.manual_seed(N + K + M)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    S = int(C.bf16_ring_splits(N, K))
    assert S > 1
    part = C.gemm_bf16_ring(x, ops.pack_bf16_weight(w), b, N, 3, S)
    assert part.shape == (S, M, N) and part.dtype == torch.float32
    ref = x.float() @ w.float().t() + b.float()
    _close(part.sum(0), ref, 1e-2, 1e-3)

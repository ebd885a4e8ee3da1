"""129-256-row decode GEMMs (gemm_i8.hip ``launch_rows256``: ring2 with the rows split in two
halves that stream one weight panel on the same XCD) against the fp32 reference ops.

One 256-row decode micro-batch reads every weight from HBM once per step, where two 128-row
lanes read it twice.  Every geometry the launcher can pick (``tune("ring2_256", cfg, nt)``) and
both weight cache policies are covered: whole-K bf16 outputs (qkv), split-K fp32 partial slices
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


def _tuned(C, cfg, nt):
    class _Ctx:
        def __enter__(self):
            C.tune("ring2_256", cfg, nt)

        def __exit__(self, *a):
            C.tune("ring2_256", 0, 1)
            return False
    return _Ctx()


@pytest.mark.parametrize("cfg,nt", [(0, 0), (0, 1), (1, 1), (2, 1), (3, 1)])
@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("N,K", [(12288, 4096), (6144, 4096), (4096, 4096), (2560, 2560)])
def test_rows256_out(cuda, cfg, nt, M, N, K):
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
    with _tuned(C, cfg, nt):
        out = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
        again = C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
    assert torch.equal(out, again)
    _close(out, ref, 1e-2, 1e-2)


@pytest.mark.parametrize("cfg,nt", [(0, 0), (0, 1), (1, 1), (2, 1), (3, 1)])
@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("grouped,magic", [(True, 1), (True, 0), (False, 1)])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (1024, 14336)])
def test_rows256_splitk(cuda, cfg, nt, M, grouped, magic, N, K):
    """Split-K slices vs the fp32 reference.  Grouped scales, default geometry: the one-VALU
    magic-number fold (gemm_i8.hip DT = 2) rounds within 8 biased terms per accumulator, so it is
    held to 1e-4 of the output's largest magnitude (measured 4.2-4.7e-5); the exact cvt + fma
    fold (magic 0) and every other form to the exact-integer tolerance."""
    C = ops.ext()
    C.tune("ring2_256_magic", magic, 0)
    torch.manual_seed(M * 7 + K)
    Mpad = (M + 15) // 16 * 16
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = (torch.rand(K // 64, Mpad, device=cuda) if grouped else torch.rand(M, device=cuda)) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    try:
        with _tuned(C, cfg, nt):
            parts = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, 0)
            again = C.w8a8_gemm_splitk(qx, sx, wp, sw, bias, N, K, 0)
    finally:
        C.tune("ring2_256_magic", 1, 0)
    S = 4 if K // 128 >= 64 else 2
    assert parts.shape == (S, M, N)
    assert torch.equal(parts, again)
    ref = _ref.w8a8_linear(qx, sx, w, sw, bias, torch.float32)
    atol = max(1e-3, 1e-4 * ref.abs().max().item()) if grouped and magic and cfg == 0 else 1e-3
    _close(parts.sum(0), ref, atol, 1e-2)


@pytest.mark.parametrize("cfg,nt", [(0, 0), (0, 1), (1, 1), (2, 1), (3, 1), (5, 1)])
@pytest.mark.parametrize("M", [129, 256])
@pytest.mark.parametrize("F,K", [(11008, 4096), (14336, 4096), (1024, 2048)])
def test_rows256_gluq(cuda, cfg, nt, M, F, K):
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
    with _tuned(C, cfg, nt):
        q, s = C.w8a8_gemm_gluq(qx, sx, wp, swb, bb, 2 * F, K)
    Mpad = (M + 15) // 16 * 16
    assert s.shape == (F // 64, Mpad)
    assert (s[:, M:] == 0).all()
    step = s[:, :M].t().unsqueeze(-1)
    deq = q.float().view(M, F // 64, 64) * step
    err = (deq - ref.float().view(M, F // 64, 64)).abs()
    assert (err <= 0.51 * step + 1e-2 * ref.float().view(M, F // 64, 64).abs() + 1e-3).all(), err.max().item()


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("kind,N,K", [("out", 12288, 4096), ("out", 2560, 2560), ("gluq", 22016, 4096),
                                      ("gluq", 2048, 2048)])
def test_rows256_restaged_epilogue_bitexact(cuda, M, kind, N, K):
    """The restaged 16-B store epilogue (tune ring2_256_rst 1, default) writes the same bits as the
    direct per-fragment stores (rst 0), including the ragged last rows of the upper half."""
    C = ops.ext()
    torch.manual_seed(M + N)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(M, device=cuda) * 0.004 + 1e-4
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.004 + 1e-4
    bias = torch.randn(N, device=cuda).to(torch.bfloat16)
    wp = ops.pack_int8_weight(w)
    outs = []
    try:
        for rst in (0, 1):
            C.tune("ring2_256_rst", rst, 0)
            r = C.w8a8_gemm_gluq(qx, sx, wp, sw, bias, N, K) if kind == "gluq" else C.w8a8_gemm(qx, sx, wp, sw, bias, N, K)
            outs.append([t.clone() for t in r] if isinstance(r, (tuple, list)) else [r.clone()])
    finally:
        C.tune("ring2_256_rst", 1, 0)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_rows256_model_routes(cuda):
    """A W8A8 Llama layer stack at 256 decode rows takes the fused path: grouped-scale attention
    output, split-K o / down partials, quantising GLU (decode_rows_ok routes 129-256 rows)."""
    assert ops.decode_rows_ok(256, 4096) and ops.decode_rows_ok(256, 11008, 4)
    assert not ops.decode_rows_ok(257, 4096)


@pytest.mark.parametrize("short,long", [(2, 2), (4, 8), (2, 8)])
@pytest.mark.parametrize("M", [129, 256])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008)])
def test_rows256_splitk_slice_counts(cuda, short, long, M, N, K):
    """Every slice count the ``ring2_256_splits=short,long`` knob selects (uneven stage splits
    included: 86 stages in 8 slices) sums to the fp32 reference."""
    C = ops.ext()
    torch.manual_seed(M + K + long)
    Mpad = (M + 15) // 16 * 16
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=cuda)
    sx = torch.rand(K // 64, Mpad, device=cuda) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=cuda)
    sw = torch.rand(N, device=cuda) * 0.01 + 1e-3
    wp = ops.pack_int8_weight(w)
    try:
        C.tune("ring2_256_splits", short, long)
        parts = C.w8a8_gemm_splitk(qx, sx, wp, sw, None, N, K, 0)
    finally:
        C.tune("ring2_256_splits", 2, 0)
    assert parts.shape == (long if K // 128 >= 64 else short, M, N)
    ref = _ref.w8a8_linear(qx, sx, w, sw, None, torch.float32)
    _close(parts.sum(0), ref, max(1e-3, 1e-4 * ref.abs().max().item()), 1e-2)

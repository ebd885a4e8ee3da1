"""fp16 execution path (the reference's fp16 agents: Code/Base Models/phi2-pythia_fp_updated.py:32,
combine_model_fp_updated.py:32-34): every fp16 kernel instantiation against the fp32 PyTorch
reference (ops/_ref.py) of the same fp16 inputs, then whole fp16 models (HIP path vs the reference
path on the same weights, graph-captured decode vs eager).

The kernels are called through ``edgellm.ops.ext()`` with fp16 tensors, so a missing fp16
instantiation fails loudly (the bindings reject dtypes they do not run)."""
import math

import pytest
import torch

from edgellm import ops
from edgellm.ops import _ref

pytestmark = pytest.mark.gpu
H16 = torch.float16


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad} / {a.numel()} elements off, max err {err.max().item():.4g}"


@pytest.mark.parametrize("H", [768, 2048, 2560, 5120])
@pytest.mark.parametrize("rms", [True, False])
@pytest.mark.parametrize("with_res", [False, True])
def test_norm_fp16(cuda, H, rms, with_res):
    C = ops.ext()
    torch.manual_seed(0)
    x = torch.randn(9, H, device=cuda, dtype=H16)
    r = torch.randn(9, H, device=cuda, dtype=H16) if with_res else None
    w = (torch.rand(H, device=cuda) + 0.5).to(H16)
    b = None if rms else torch.randn(H, device=cuda).to(H16)
    y, _, ro = C.norm(x, r, w, b, 1e-5, rms, 0)
    yr, ror = _ref.rms_norm(x, w, 1e-5, r) if rms else _ref.layer_norm(x, w, b, 1e-5, r)
    assert y.dtype == H16 and ro.dtype == H16
    _close(y, yr, 2e-3, 2e-3)
    _close(ro, ror, 0)


@pytest.mark.parametrize("S", [1, 4])
def test_rms_norm_parts_fp16(cuda, S):
    """Split-K fp32 slices summed in order, rounded to fp16, (+ residual), normalised."""
    C = ops.ext()
    M, H = 3, 2048
    parts = torch.randn(S, M, H, device=cuda)
    res = torch.randn(M, H, device=cuda).to(H16)
    w = (torch.rand(H, device=cuda) + 0.5).to(H16)
    y, s, h = C.rms_norm_parts(parts, res, w, 1e-5, 0)
    acc = parts[0].clone()
    for i in range(1, S):
        acc += parts[i]
    yr, hr = _ref.rms_norm(acc.to(H16), w, 1e-5, res)
    assert s is None and y.dtype == H16
    _close(h, hr, 0)
    _close(y, yr, 2e-3, 2e-3)


@pytest.mark.parametrize("mode,act", [(0, "silu_glu"), (1, "gelu_tanh"), (2, "gelu")])
def test_act_embedding_maxprob_fp16(cuda, mode, act):
    C = ops.ext()
    F = 2560
    W = 2 * F if mode == 0 else F
    x = (torch.randn(5, W, device=cuda) * 2).to(H16)
    y, _ = C.act(x, mode, False)
    yr = _ref.silu_mul(x) if mode == 0 else _ref.gelu(x, "tanh" if mode == 1 else "none")
    _close(y, yr, 2e-3, 2e-3)
    table = torch.randn(1000, 256, device=cuda).to(H16)
    ids = torch.randint(0, 1000, (3, 5), device=cuda)
    assert torch.equal(C.embedding(ids, table, False), table[ids])
    assert torch.equal(C.embedding(ids, table, True), table[ids].float())
    logits = (torch.randn(4, 50304, device=cuda) * 3).to(H16)
    _close(C.max_prob(logits), _ref.max_softmax_prob(logits), 1e-6, 1e-4)


@pytest.mark.parametrize("Hq,Hkv,D,rot", [(32, 32, 80, 32), (8, 8, 256, 64), (32, 8, 64, 64)])
def test_rope_kv_write_fp16(cuda, Hq, Hkv, D, rot):
    C = ops.ext()
    B, T, S = 3, 5, 64
    qkv = torch.randn(B * T, (Hq + 2 * Hkv) * D, device=cuda).to(H16)
    start = torch.tensor([0, 7, 30], device=cuda, dtype=torch.int32)
    rope = _ref.rope_tables(rot, S, 10000.0, device=cuda)
    kc = torch.zeros(B, Hkv, S, D, device=cuda, dtype=H16)
    vc = torch.zeros_like(kc)
    kr, vr = kc.clone(), vc.clone()
    q = C.rope_kv_write(qkv, start, rope, kc, vc, Hq, Hkv, D, rot)
    qr = _ref.rope_kv_write(qkv, start, rope, kr, vr, Hq, Hkv, D, rot)
    assert q.dtype == H16
    _close(q, qr, 2e-3, 2e-3)
    _close(kc, kr, 2e-3, 2e-3)
    assert torch.equal(vc, vr)
    with pytest.raises(RuntimeError):              # mixed dtypes are refused, not reinterpreted
        C.rope_kv_write(qkv, start, rope, kc.bfloat16(), vc.bfloat16(), Hq, Hkv, D, rot)


@pytest.mark.parametrize("Hq,Hkv,D", [(32, 32, 80), (8, 8, 256), (32, 8, 128), (16, 16, 64)])
@pytest.mark.parametrize("lens", [(1, 17, 200), (4096, 1000, 3333)])
def test_decode_attention_fp16(cuda, Hq, Hkv, D, lens):
    C = ops.ext()
    B = len(lens)
    S = max(lens) + 5
    q = torch.randn(B, Hq, D, device=cuda).to(H16)
    kc = torch.randn(B, Hkv, S, D, device=cuda).to(H16)
    vc = torch.randn(B, Hkv, S, D, device=cuda).to(H16)
    sl = torch.tensor(lens, device=cuda, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    out = C.decode_attn(q, kc, vc, sl, scale, max(lens))
    ref = _ref.decode_attention(q, kc, vc, sl, scale)
    assert out.dtype == H16
    _close(out, ref, 3e-3, 5e-3)


@pytest.mark.parametrize("occ", [4, 0])
@pytest.mark.parametrize("Hq,Hkv,D,rot", [(32, 32, 80, 32), (8, 8, 256, 64), (32, 8, 128, 128)])
def test_decode_attention_fused_fp16(cuda, occ, Hq, Hkv, D, rot):
    """RoPE on q + KV append + attention in one launch, against rope_kv_write + decode_attn."""
    C = ops.ext()
    B, S = 5, 300
    lens = torch.tensor([1, 9, 120, 299, 64], device=cuda, dtype=torch.int32)
    pos = lens - 1
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=cuda).to(H16)
    kc = torch.randn(B, Hkv, S, D, device=cuda).to(H16)
    vc = torch.randn(B, Hkv, S, D, device=cuda).to(H16)
    kr, vr = kc.clone(), vc.clone()
    rope = _ref.rope_tables(rot, S, 10000.0, device=cuda)
    scale = 1 / math.sqrt(D)
    try:
        C.tune("decode_attn_occ", occ, 0)
        out, s = C.decode_attn_fused(qkv, pos, rope, kc, vc, lens, Hq, scale, S, rot, False)
    finally:
        C.tune("decode_attn_occ", 4, 0)
    q = _ref.rope_kv_write(qkv, pos, rope, kr, vr, Hq, Hkv, D, rot)
    ref = _ref.decode_attention(q.view(B, Hq, D), kr, vr, lens, scale)
    assert s is None and out.dtype == H16
    _close(kc, kr, 2e-3, 2e-3)
    assert torch.equal(vc, vr)
    _close(out, ref, 3e-3, 5e-3)
    with pytest.raises(RuntimeError):              # no int8 output from fp16 rows
        C.decode_attn_fused(qkv, pos, rope, kc, vc, lens, Hq, scale, S, rot, True)


@pytest.mark.parametrize("fa", [0, 2])
@pytest.mark.parametrize("Hq,Hkv,D", [(32, 32, 80), (8, 8, 256), (8, 2, 128), (16, 16, 64)])
@pytest.mark.parametrize("T,starts", [(100, (0, 37)), (300, (0, 0))])
def test_prefill_attention_fp16(cuda, fa, Hq, Hkv, D, T, starts):
    """fp16 MFMA prefill: the 16-row kernel (every D) and the LDS-DMA fa_kernel (D 64 / 128)."""
    C = ops.ext()
    B = len(starts)
    S = max(starts) + T + 3
    q = torch.randn(B, T, Hq, D, device=cuda).to(H16)
    kc = torch.randn(B, Hkv, S, D, device=cuda).to(H16)
    vc = torch.randn(B, Hkv, S, D, device=cuda).to(H16)
    sp = torch.tensor(starts, device=cuda, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    try:
        C.tune("prefill_fa", fa, 0)
        out = C.prefill_attn(q, kc, vc, sp, scale, True)
    finally:
        C.tune("prefill_fa", 1, 0)
    ref = _ref.prefill_attention(q, kc, vc, sp, scale, True)
    assert out.dtype == H16
    _close(out, ref, 3e-3, 5e-3)


@pytest.mark.parametrize("epi,act", [(0, None), (1, "silu_glu"), (2, "gelu_tanh"), (3, "gelu")])
@pytest.mark.parametrize("M", [1, 5, 16, 40])
@pytest.mark.parametrize("N,K", [(2560, 2560), (10240, 2560), (2048, 8192)])
def test_gemv_fp16(cuda, epi, act, M, N, K):
    C = ops.ext()
    torch.manual_seed(1)
    x = torch.randn(M, K, device=cuda).to(H16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(H16)
    bias = (torch.randn(N, device=cuda) * 0.1).to(H16)
    y = C.gemv_bf16(x, ops.pack_bf16_weight(w), bias, N, epi, None)
    lin = (x.float() @ w.float().t() + bias.float()).to(H16)      # the GEMM output rounds to fp16
    if epi == 0:
        ref = lin
    elif epi == 1:
        ref = _ref.silu_mul(lin)
    else:
        ref = _ref.gelu(lin, "tanh" if epi == 2 else "none")
    assert y.dtype == H16
    _close(y, ref, 4e-3, 4e-3)
    if epi == 0:
        add = torch.randn(M, N, device=cuda).to(H16)
        y2 = C.gemv_bf16(x, ops.pack_bf16_weight(w), bias, N, 0, add)
        _close(y2, (lin.float() + add.float()).to(H16), 8e-3, 4e-3)
        part = C.gemv_bf16_splitk(x, ops.pack_bf16_weight(w), bias, N, 4)
        _close(part.sum(0), x.float() @ w.float().t() + bias.float(), 2e-3, 2e-3)


def test_linear_fp16_routes_to_gemv(cuda):
    """ops.linear_bf16 on fp16 decode rows runs the fp16 GEMV (mode 1); 17+ rows go to hipBLASLt
    (the ring GEMM is bf16-only); a dtype mismatch never reaches a kernel."""
    x = torch.randn(4, 2560, device=cuda).to(H16)
    w = torch.randn(2560, 2560, device=cuda).to(H16)
    assert ops.bf16_decode_mode(x, w) == 1
    assert ops.bf16_decode_mode(torch.randn(64, 2560, device=cuda).to(H16), w) == 0
    assert ops.bf16_decode_mode(x, w.bfloat16()) == 0
    _close(ops.linear_bf16(x, w), (x.float() @ w.float().t()).to(H16), 0.5, 4e-3)


def test_sampler_fp16_logits(cuda):
    """fp16 logits are widened to fp32 before the fused sampler: same tokens as fp32 logits."""
    lg = (torch.randn(3, 32000, device=cuda) * 4).to(H16)
    rng = torch.tensor([7, 0], dtype=torch.int32, device=cuda)
    a = ops.sample(lg, None, 0.7, 50, 0.9, 1.0, rng.clone())
    b = ops.sample(lg.float(), None, 0.7, 50, 0.9, 1.0, rng.clone())
    assert torch.equal(a, b)


def _logits(model, ids, dev):
    from edgellm.engine import KVCache
    from edgellm.models import AttnCtx
    B, T = ids.shape
    kv = KVCache(model.cfg, B, T + 1, dtype=model.dtype, device=dev)
    sp = torch.zeros(B, dtype=torch.int32, device=dev)
    ctx = AttnCtx("prefill", B, T, sp, sp + T, T, kv, model.rope_table(dev))
    return model(ids, ctx, logits="all").float()


@pytest.mark.parametrize("arch", ["phi", "gpt_neox", "llama", "gpt2"])
def test_fp16_model_matches_reference_path(cuda, arch, monkeypatch):
    from edgellm.models import build_model, tiny
    ops.ext()
    cfg = tiny(arch)
    m = build_model(cfg, dtype=H16, device=cuda, seed=4)
    assert m.dtype == H16
    ids = torch.randint(0, cfg.vocab_size, (2, 37), device=cuda)
    hip = _logits(m, ids, cuda)
    monkeypatch.setattr(ops, "_REF_ON_GPU", True)
    ref = _logits(m, ids, cuda)
    monkeypatch.setattr(ops, "_REF_ON_GPU", False)
    rel = ((hip - ref).norm() / ref.norm()).item()
    assert rel < 8e-3, rel


@pytest.mark.parametrize("arch", ["phi", "gpt_neox", "llama"])
def test_fp16_decode_graph_equals_eager(cuda, arch):
    """fp16 decode steps (fp16 GEMV, fused fp16 attention, fp16 norms) captured in graphs give the
    eager tokens, and greedy tokens match the reference path's."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    m = build_model(tiny(arch, num_layers=3), dtype=H16, device=cuda, seed=2)
    prompts = [[5, 9, 2, 44, 17, 3], [8, 1, 77, 4, 12, 6]]
    sp = SamplingParams(max_new_tokens=30, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)
    g1 = Generator(m, max_batch=2, max_seq=200, use_graphs=True).generate(prompts, sp, seed=3)
    g2 = Generator(m, max_batch=2, max_seq=200, use_graphs=False).generate(prompts, sp, seed=3)
    assert g1.tokens == g2.tokens


def test_precision_dtype_honours_fp16(cuda):
    from edgellm.models.registry import precision_dtype
    assert precision_dtype("fp16", cuda) == H16
    assert precision_dtype("bf16", cuda) == torch.bfloat16
    assert precision_dtype("fp16", cuda, "w8a8_smoothquant") == torch.bfloat16


@pytest.mark.parametrize("mode", ["w8a8_smoothquant", "llm_int8"])
def test_int8_checkpoint_with_fp16_precision(cuda, tmp_path, mode):
    """An INT8 checkpoint loaded with the reference's fp16 precision runs bf16 activations (the
    INT8 kernels' epilogues and the quantising norm take bf16) and decodes on the GPU."""
    from edgellm.cli import quantize
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models.registry import load_model
    out = quantize.main(["--model", "tiny:llama", "--quant", mode, "--out", str(tmp_path / "ck"),
                         "--precision", "bf16", "--device", "cpu"])
    m, _, source = load_model(out, "fp16", "none", cuda)
    assert source.startswith("int8-checkpoint:") and m.dtype == torch.bfloat16
    res = Generator(m, max_batch=1, max_seq=64).generate([[3, 1, 4, 1, 5, 9]], SamplingParams(max_new_tokens=6),
                                                         seed=0)
    assert len(res.tokens[0]) == 6


@pytest.mark.parametrize("arch", ["llama", "gpt_neox"])
def test_fp16_model_with_int8_kv_falls_back(cuda, arch):
    """--precision fp16 --kv_dtype int8: the int8-KV kernels take bf16 q / k / v, so an fp16
    model gets a 16-bit cache (logged) instead of failing at prefill; the tokens equal the
    bf16-KV run's."""
    from edgellm.cli.common import build_generator
    from edgellm.engine import SamplingParams
    from edgellm.models import build_model, tiny
    from edgellm.offload import HeadInferKV
    m = build_model(tiny(arch, num_layers=2), dtype=H16, device=cuda, seed=1)
    g8 = build_generator(m, dict(max_seq=96, kv_dtype="int8"), max_batch=2)
    assert not g8.kv.quantized and g8.kv.k.dtype == H16
    sp = SamplingParams(max_new_tokens=8, do_sample=False)
    prompts = [[5, 9, 2, 44, 17, 3], [8, 1, 77, 4, 12, 6]]
    g16 = build_generator(m, dict(max_seq=96, kv_dtype="bf16"), max_batch=2)
    assert g8.generate(prompts, sp, seed=0).tokens == g16.generate(prompts, sp, seed=0).tokens
    hi = HeadInferKV(m.cfg, 1, 64, 0, cuda, dtype=H16, kv_dtype="int8")
    assert not hi.q8

"""int8 KV cache (engine.kv_cache kv_dtype="int8"; ops/csrc/attn_decode_i8.hip).

CPU: the reference semantics — per-(token, head) quantisation of the rotated k / v rows, decode
and prefill through the int8 cache — stay close to the bf16-cache model, and the cache holds
exactly quant_kv_rows of the resident cache's rows.
GPU: the fused decode kernel (RoPE + quantising append + attention, split and direct forms,
int8-output form) and the prefill append kernel against the fp32 reference.
"""
import pytest
import torch

import edgellm  # noqa: F401
from edgellm import ops
from edgellm.engine import Generator, SamplingParams
from edgellm.engine.kv_cache import KVCache
from edgellm.models import build_model, tiny
from edgellm.ops import _ref


def _cfg(arch="llama", D=64, layers=2):
    if arch == "llama":     # GQA 2:1
        return tiny("llama", hidden_size=2 * D, num_heads=2, num_kv_heads=1, num_layers=layers)
    return tiny("llama2", hidden_size=2 * D, num_heads=2, num_kv_heads=2, num_layers=layers)


@pytest.mark.parametrize("arch", ["llama", "llama2"])
def test_kv_int8_generate_close_to_bf16_cache_cpu(arch):
    cfg = _cfg(arch)
    m = build_model(cfg, dtype=torch.float32, seed=3)
    prompts = torch.randint(0, cfg.vocab_size, (3, 11), generator=torch.Generator().manual_seed(1)).tolist()
    sp = SamplingParams(max_new_tokens=6, do_sample=False)
    g16 = Generator(m, max_batch=3, max_seq=32)
    g8 = Generator(m, max_batch=3, max_seq=32, kv_dtype="int8")
    assert g8.kv.quantized and g8.kv.k.dtype == torch.int8
    r16 = g16.generate(prompts, sp)
    r8 = g8.generate(prompts, sp)
    # the int8 cache holds exactly the quantised rows of the resident cache (11 prompt + 5 decoded)
    for li in range(cfg.num_layers):
        k16, v16 = g16.kv.layer(li)
        k8, v8 = g8.kv.layer(li)
        ks, vs = g8.kv.layer_scales(li)
        n = 11
        q, s = _ref.quant_kv_rows(k16[:, :, :n])
        if li == 0:                     # layer 0 sees identical inputs on the prompt: bit-exact cache
            assert torch.equal(k8[:, :, :n], q) and torch.allclose(ks[:, :, :n], s)
            deq = _ref.dequant_kv(k8[:, :, :n], ks[:, :, :n])
            assert ((deq - k16[:, :, :n]).abs() <= 0.5001 * ks[:, :, :n, None]).all()
        deq = _ref.dequant_kv(k8[:, :, :n], ks[:, :, :n])
        assert (deq - k16[:, :, :n]).norm() / k16[:, :, :n].norm() < 0.05
    agree = sum(a == b for x, y in zip(r16.tokens, r8.tokens) for a, b in zip(x, y)) / sum(map(len, r16.tokens))
    assert agree >= 0.8, (r16.tokens, r8.tokens)


def test_kv_int8_logits_close_cpu():
    cfg = _cfg("llama2", D=64)
    m = build_model(cfg, dtype=torch.float32, seed=5)
    ids = torch.randint(0, cfg.vocab_size, (2, 9), generator=torch.Generator().manual_seed(2))
    outs = {}
    for kvd in ("bf16", "int8"):
        g = Generator(m, max_batch=2, max_seq=32, kv_dtype=kvd)
        g.prefill(ids[:, :6])
        outs[kvd] = g.prefill(ids[:, 6:], 0, 6)     # chunk with history: int8 dequantises the prefix
    ref, got = outs["bf16"], outs["int8"]
    rel = (got - ref).norm() / ref.norm()
    assert rel < 0.05, rel


def test_kv_int8_falls_back_for_head_dim():
    kv = KVCache(tiny("phi"), 1, 8, kv_dtype="int8")     # head_dim 80: no int8 kernels -> 16-bit cache
    assert not kv.quantized and kv.k.dtype == torch.bfloat16


# --------------------------------------------------------------------------- GPU kernels
def _decode_case(dev, B, Hq, Hkv, D, S, lens, quant_out, seed=0, wave=False):
    g = torch.Generator().manual_seed(seed)
    qkv = (torch.randn(B, (Hq + 2 * Hkv) * D, generator=g)).to(torch.bfloat16)
    k = torch.randn(B, Hkv, S, D, generator=g)
    v = torch.randn(B, Hkv, S, D, generator=g)
    kq, ks = _ref.quant_kv_rows(k)
    vq, vs = _ref.quant_kv_rows(v)
    seq_lens = torch.tensor(lens, dtype=torch.int32)
    pos = seq_lens - 1
    rope = _ref.rope_tables(D, S + 8, 10000.0)
    args_cpu = [qkv, pos, rope, kq.clone(), vq.clone(), ks.clone(), vs.clone(), seq_lens]
    args_gpu = [t.to(dev) for t in args_cpu]
    ref = ops.decode_attention_fused_i8(*args_cpu, Hq, D ** -0.5, S, D, quant_out)
    # wave=True: enable the wave-per-(sequence, head) kernel (off by default; tune key
    # attn8_wave_max = longest cache it takes) for this call only
    if wave:
        ops.ext().tune("attn8_wave_max", S, 0)
    try:
        got = ops.decode_attention_fused_i8(*args_gpu, Hq, D ** -0.5, S, D, quant_out)
        torch.cuda.synchronize()
    finally:
        if wave:
            ops.ext().tune("attn8_wave_max", 0, 0)
    return args_cpu, args_gpu, ref, got


@pytest.mark.gpu
@pytest.mark.parametrize("B,Hq,Hkv,D,S,lens,wave", [
    (3, 4, 4, 128, 160, [160, 97, 1], False),         # MHA (Llama-2-7B heads), one split
    (2, 8, 2, 128, 3000, [3000, 1500], False),        # GQA 4:1, split-K + combine
    (2, 4, 1, 64, 700, [700, 65], False),             # D = 64, GQA 4:1
    (1, 2, 2, 256, 300, [300], False),                # D = 256
    (64, 32, 32, 128, 200, [200 - 3 * i for i in range(64)], False),   # workgroup form at B*H >= 2048
    (64, 32, 32, 128, 200, [200 - 3 * i for i in range(64)], True),    # wave-per-head form
    (128, 16, 16, 64, 90, [90 - (i % 89) for i in range(128)], True),  # wave form, D = 64, lens down to 2
])
def test_decode_attn_i8_kernel_vs_ref(cuda, B, Hq, Hkv, D, S, lens, wave):
    cpu, gpu, ref, got = _decode_case(cuda, B, Hq, Hkv, D, S, lens, False, wave=wave)
    out_r, out_g = ref[0].float(), got[0].float().cpu()
    err = (out_g - out_r).abs().max().item()
    assert err < 2e-2, err
    # the appended row: int8 within one step of the reference rounding, scales within bf16 rounding
    for cache_c, cache_g, sc_c, sc_g in ((cpu[3], gpu[3], cpu[5], gpu[5]), (cpu[4], gpu[4], cpu[6], gpu[6])):
        for b, L in enumerate(lens):
            p = L - 1
            dq = (cache_g[b, :, p].cpu().int() - cache_c[b, :, p].int()).abs()
            assert dq.max() <= 1
            assert torch.allclose(sc_g[b, :, p].cpu(), sc_c[b, :, p], rtol=1e-2)


@pytest.mark.gpu
def test_decode_attn_i8_quant_out(cuda):
    cpu, gpu, ref, got = _decode_case(cuda, 4, 8, 8, 128, 200, [200, 150, 90, 3], True, seed=1)
    deq_r = ref[0].float().view(4, -1, 64) * ref[1][:, :4].t().reshape(4, -1, 1)
    deq_g = got[0].float().cpu().view(4, -1, 64) * got[1][:, :4].cpu().t().reshape(4, -1, 1)
    assert (deq_g - deq_r).abs().max() < 3e-2


@pytest.mark.gpu
def test_decode_attn_i8_quant_out_wave(cuda):
    """The wave-per-(sequence, head) kernel's quantised-output branch (per-(token, 64) o input)."""
    B = 64
    lens = [200 - 3 * i for i in range(B)]
    cpu, gpu, ref, got = _decode_case(cuda, B, 32, 32, 128, 200, lens, True, seed=2, wave=True)
    G = ref[0].shape[1] // 64
    deq_r = ref[0].float().view(B, G, 64) * ref[1][:, :B].t().reshape(B, G, 1)
    deq_g = got[0].float().cpu().view(B, G, 64) * got[1][:, :B].cpu().t().reshape(B, G, 1)
    assert (deq_g - deq_r).abs().max() < 3e-2


@pytest.mark.gpu
@pytest.mark.parametrize("D", [64, 128, 256])
def test_kv_quant_append_kernel(cuda, D):
    B, Hkv, S, T = 3, 2, 40, 7
    g = torch.Generator().manual_seed(D)
    src = torch.randn(B, Hkv, S, D, generator=g).to(torch.bfloat16)
    start = torch.tensor([0, 5, 30], dtype=torch.int32)
    c_r = torch.zeros(B, Hkv, S, D, dtype=torch.int8)
    s_r = torch.zeros(B, Hkv, S)
    ops.kv_quant_append(src, start, T, c_r, s_r)
    c_g, s_g = c_r.zero_().clone().to(cuda), s_r.zero_().clone().to(cuda)
    ops.kv_quant_append(src, start, T, c_r, s_r)
    ops.kv_quant_append(src.to(cuda), start.to(cuda), T, c_g, s_g)
    torch.cuda.synchronize()
    # bit-exact up to a rounding tie: at most one step on at most 0.1 % of the values
    d = (c_g.cpu().int() - c_r.int()).abs()
    assert d.max() <= 1 and (d > 0).float().mean() < 1e-3
    assert torch.allclose(s_g.cpu(), s_r)


@pytest.mark.gpu
def test_generate_int8_kv_gpu_close_to_bf16(cuda):
    """Model-level: Llama-2-geometry heads (D = 128), W8A8, graph-captured decode over the int8
    cache against the same model over the bf16 cache: decode logits within 5 % relative."""
    from edgellm.quant import quantize_model
    cfg = tiny("llama2", hidden_size=256, num_heads=2, num_kv_heads=2, num_layers=2, intermediate_size=512)
    m = quantize_model(build_model(cfg, device=cuda, seed=0), "w8a8")
    ids = torch.randint(0, cfg.vocab_size, (4, 20), generator=torch.Generator().manual_seed(0)).to(cuda)
    logits = {}
    for kvd in ("bf16", "int8"):
        g = Generator(m, max_batch=4, max_seq=64, kv_dtype=kvd)
        g.prefill(ids[:, :19])
        logits[kvd] = g.prefill(ids[:, 19:], 0, 19).float()
    rel = ((logits["int8"] - logits["bf16"]).norm() / logits["bf16"].norm()).item()
    assert rel < 0.05, rel
    sp = SamplingParams(max_new_tokens=12, do_sample=False)
    r16 = Generator(m, max_batch=4, max_seq=64).generate(ids.tolist(), sp)
    r8 = Generator(m, max_batch=4, max_seq=64, kv_dtype="int8").generate(ids.tolist(), sp)
    assert all(len(t) == 12 for t in r8.tokens)
    agree = sum(a == b for x, y in zip(r16.tokens, r8.tokens) for a, b in zip(x, y)) / 48
    assert agree >= 0.7, agree


@pytest.mark.gpu
@pytest.mark.parametrize("D", [64, 128, 256])
def test_kv_dequant_kernel(cuda, D):
    """int8 cache rows -> bf16 scratch (chunked-prefill history) == the fp32 reference rounded once."""
    B, Hkv, S, T = 3, 2, 40, 29
    g = torch.Generator().manual_seed(D + 1)
    c = torch.randint(-127, 128, (B, Hkv, S, D), generator=g, dtype=torch.int8)
    s = torch.rand(B, Hkv, S, generator=g) * 0.05
    ref = (c[:, :, :T].float() * s[:, :, :T, None]).to(torch.bfloat16)
    dst = torch.zeros(B, Hkv, S + 3, D, dtype=torch.bfloat16, device=cuda)
    ops.kv_dequant(c.to(cuda), s.to(cuda), dst, T)
    torch.cuda.synchronize()
    assert torch.equal(dst[:, :, :T].cpu(), ref)
    assert (dst[:, :, T:] == 0).all()


def test_prefill_scratch_reused_across_layers():
    """KVCache.prefill_scratch: one grow-only buffer per stream, views of the requested shape."""
    from edgellm.engine import KVCache
    cfg = tiny("llama2", hidden_size=256, num_heads=2, num_kv_heads=2, num_layers=2, intermediate_size=512)
    kv = KVCache(cfg, 4, 64, kv_dtype="int8")
    k1, v1 = kv.rows(0, 2).prefill_scratch(2, 30, torch.bfloat16, "cpu")
    assert k1.shape == (2, 2, 30, cfg.head_dim) and k1.is_contiguous() and v1.is_contiguous()
    k2, _ = kv.prefill_scratch(2, 20, torch.bfloat16, "cpu")
    assert k2.data_ptr() == k1.data_ptr()                    # smaller request: same storage
    k3, _ = kv.prefill_scratch(4, 64, torch.bfloat16, "cpu")
    assert k3.shape == (4, 2, 64, cfg.head_dim)

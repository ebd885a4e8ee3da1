"""HeadInfer offload: with a tiny GPU budget (H_on = 0 or 1 KV head resident) generation must be
identical to the fully-resident cache.  CPU path here; the GPU variant
(pinned pool, side-stream copies, native hipMemcpy2DAsync) is marked gpu."""
import pytest
import torch

from edgellm.engine import Generator, SamplingParams
from edgellm.models import build_model, tiny
from edgellm.offload import HeadInferKV, heads_for_budget


def _run(device, h_on, chunk_heads, chunk_size, kvh=4, arch="llama", dtype=torch.float32, T=23, new=9):
    cfg = tiny(arch, num_kv_heads=kvh, num_heads=8, hidden_size=128, num_layers=3)
    m = build_model(cfg, dtype=dtype, device=device, seed=9)
    prompts = [[(7 * i + 3 * b) % cfg.vocab_size for i in range(T)] for b in range(2)]
    sp = SamplingParams(max_new_tokens=new, temperature=0.8, top_k=20, top_p=0.95, repetition_penalty=1.1)
    # same chunked prefill on both sides: only the offload differs (chunking changes bf16 GEMM shapes)
    ref = Generator(m, max_batch=2, max_seq=64, use_graphs=False, prefill_chunk=chunk_size).generate(prompts, sp,
                                                                                                   seed=4)
    kv = HeadInferKV(cfg, 2, 64, h_on=h_on, device=device, chunk_heads=chunk_heads, chunk_size=chunk_size,
                     dtype=dtype)
    got = Generator(m, max_batch=2, max_seq=64, kv=kv).generate(prompts, sp, seed=4)
    return ref, got, kv


@pytest.mark.parametrize("h_on,chunk_heads,chunk_size", [(1, 1, 8), (0, 2, 64), (2, 1, 5), (3, 4, 16), (1, None, 8)])
def test_headinfer_matches_resident_cpu(h_on, chunk_heads, chunk_size):
    ref, got, kv = _run("cpu", h_on, chunk_heads, chunk_size)
    assert got.tokens == ref.tokens
    assert kv.bytes_d2h > 0 and kv.bytes_h2d > 0


def test_budget_to_heads():
    from edgellm.models import get_config
    cfg = get_config("llama-3-8b")
    per_head = 2 * 1 * 1_000_000 * 128 * 2 * 32
    assert heads_for_budget(cfg, 1, 1_000_000, 3 * per_head) == 3
    assert heads_for_budget(cfg, 1, 1_000_000, 10 ** 15) == cfg.num_kv_heads


@pytest.mark.gpu
@pytest.mark.parametrize("h_on,chunk_heads,chunk_size", [(1, 1, 8), (0, 2, 64), (2, 1, 5), (1, None, 8)])
def test_headinfer_matches_resident_gpu(cuda, h_on, chunk_heads, chunk_size):
    ref, got, kv = _run(cuda, h_on, chunk_heads, chunk_size, dtype=torch.bfloat16)
    assert got.tokens == ref.tokens
    assert kv.host_k.is_pinned()


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 37])
def test_copy_head_block_kernel_both_directions(cuda, T):
    """offload.hip::head_block_copy_kernel: strided [B, c, T, D] blocks between a pinned host pool
    and a device buffer, against torch's copy of the same views (bit-exact)."""
    from edgellm import ops
    B, H, S, D, h0, c, p0 = 5, 8, 64, 128, 3, 4, 9
    for mode, want in ((0, "kernel"), (1, "kernel"), (2, "dma")):
        host = torch.randn(B, H, S, D, dtype=torch.bfloat16).pin_memory()
        dev = torch.zeros(B, c, S, D, dtype=torch.bfloat16, device="cuda")
        # short rows: auto picks the one-launch kernel; mode 2 forces the copy engines
        assert ops.copy_head_block(dev[:, :, p0:p0 + T], host[:, h0:h0 + c, p0:p0 + T], mode) == want
        torch.cuda.synchronize()
        assert torch.equal(dev[:, :, p0:p0 + T].cpu(), host[:, h0:h0 + c, p0:p0 + T])
        assert not dev[:, :, :p0].any() and not dev[:, :, p0 + T:].any()
        src = torch.randn(B, c, T, D, dtype=torch.bfloat16, device="cuda")
        before = host.clone()
        assert ops.copy_head_block(host[:, h0:h0 + c, p0:p0 + T], src, mode) == want
        torch.cuda.synchronize()
        before[:, h0:h0 + c, p0:p0 + T] = src.cpu()
        assert torch.equal(host, before)


@pytest.mark.gpu
def test_copy_head_block_long_rows_use_copy_engines(cuda):
    """History rows >= 64 KiB (long contexts) go to the SDMA engines in auto mode, bit-exact."""
    from edgellm import ops
    B, H, S, D = 1, 4, 1024, 128                 # 1024 positions x 256 B = 256 KiB per head row
    host = torch.randn(B, H, S, D, dtype=torch.bfloat16).pin_memory()
    dev = torch.zeros(B, 2, S, D, dtype=torch.bfloat16, device="cuda")
    assert ops.copy_head_block(dev, host[:, 1:3]) == "dma"
    torch.cuda.synchronize()
    assert torch.equal(dev.cpu(), host[:, 1:3])


@pytest.mark.gpu
def test_headinfer_long_context_matches_resident(cuda):
    """HeadInfer as a long-context mechanism: a 9K-token prompt prefilled in 2K chunks with ONE of
    two KV heads per layer on the GPU (history prefetched from pinned host memory each chunk and
    each decode step, SDMA for the long rows) decodes exactly the resident model's tokens."""
    cfg = tiny("llama2", hidden_size=256, num_heads=2, num_kv_heads=2, num_layers=2, intermediate_size=512,
               max_position_embeddings=16384)
    m = build_model(cfg, device=cuda, seed=3)
    T, new, chunk = 9000, 12, 2048
    g = torch.Generator().manual_seed(0)
    prompt = [torch.randint(0, cfg.vocab_size, (T,), generator=g).tolist()]
    sp = SamplingParams(max_new_tokens=new, do_sample=False)
    ref = Generator(m, max_batch=1, max_seq=T + new + 8, use_graphs=False, prefill_chunk=chunk).generate(prompt, sp)
    kv = HeadInferKV(cfg, 1, T + new + 8, h_on=1, device=cuda, chunk_size=chunk)
    got = Generator(m, max_batch=1, max_seq=T + new + 8, kv=kv).generate(prompt, sp)
    assert got.tokens == ref.tokens
    assert kv.transports.get("dma", 0) > 0 and kv.transports.get("kernel", 0) > 0
    assert kv.host_bytes() > 0 and kv.gpu.nbytes() == kv.host_bytes()      # 1 of 2 heads resident


# --------------------------------------------------------------------------- int8 offload
def _run_q8(device, h_on, chunk_heads, chunk_size, quant="none", T=23, new=9, dtype=torch.float32, seed=9):
    """int8 KV on every tier (HeadInferKV kv_dtype="int8") against the resident int8 cache."""
    from edgellm.quant import quantize_model
    cfg = tiny("llama", hidden_size=256, num_heads=8, num_kv_heads=4, intermediate_size=512, num_layers=2)
    m = build_model(cfg, dtype=dtype, device=device, seed=seed)
    if quant != "none":
        m = quantize_model(m, quant)
    prompts = [[(7 * i + 3 * b) % cfg.vocab_size for i in range(T)] for b in range(2)]
    sp = SamplingParams(max_new_tokens=new, temperature=0.8, top_k=20, top_p=0.95, repetition_penalty=1.1)
    ref = Generator(m, max_batch=2, max_seq=T + new + 8, use_graphs=False, prefill_chunk=chunk_size,
                    kv_dtype="int8").generate(prompts, sp, seed=4)
    kv = HeadInferKV(cfg, 2, T + new + 8, h_on=h_on, device=device, chunk_heads=chunk_heads, chunk_size=chunk_size,
                     dtype=dtype, kv_dtype="int8")
    got = Generator(m, max_batch=2, max_seq=T + new + 8, kv=kv).generate(prompts, sp, seed=4)
    return ref, got, kv


@pytest.mark.parametrize("h_on,chunk_heads,chunk_size", [(1, 1, 8), (0, 2, 64), (2, 1, 5), (3, None, 16)])
def test_headinfer_int8_matches_resident_int8_cpu(h_on, chunk_heads, chunk_size):
    ref, got, kv = _run_q8("cpu", h_on, chunk_heads, chunk_size)
    assert got.tokens == ref.tokens
    assert kv.host_k.dtype == torch.int8 and kv.host_ks.dtype == torch.float32
    # PCIe bytes per (token, head): D + 4 (int8 row + fp32 scale), not 2 D
    assert kv.bytes_d2h > 0 and kv.bytes_h2d > 0
    assert kv.host_bytes() == kv.host_kv.numel() + 4 * kv.host_s.numel()


@pytest.mark.gpu
@pytest.mark.parametrize("h_on,chunk_heads,chunk_size", [(1, 1, 8), (0, 2, 64), (2, None, 16)])
def test_headinfer_int8_matches_resident_int8_gpu(cuda, h_on, chunk_heads, chunk_size):
    ref, got, kv = _run_q8(cuda, h_on, chunk_heads, chunk_size, quant="w8a8", dtype=torch.bfloat16)
    assert got.tokens == ref.tokens
    assert kv.host_k.is_pinned() and kv.host_ks.is_pinned()


@pytest.mark.gpu
@pytest.mark.parametrize("kv_dtype", ["bf16", "int8"])
def test_headinfer_w8a8_long_context_logits_vs_resident(cuda, kv_dtype):
    """W8A8 model, 4.5K-token prompt prefilled in 1K chunks, 3 of 4 KV heads per layer offloaded
    (int8 or bf16 on every tier): the last prefill chunk's logits stay within tolerance of the same
    model over a fully resident cache of the same dtype, and 8 greedy decode tokens agree."""
    from edgellm.quant import quantize_model
    cfg = tiny("llama2", hidden_size=512, num_heads=4, num_kv_heads=4, num_layers=2, intermediate_size=1024,
               max_position_embeddings=8192)
    m = quantize_model(build_model(cfg, device=cuda, seed=5), "w8a8_smoothquant")
    T, new, chunk = 4500, 8, 1024
    g = torch.Generator().manual_seed(1)
    prompt = [torch.randint(0, cfg.vocab_size, (T,), generator=g).tolist()]
    sp = SamplingParams(max_new_tokens=new, do_sample=False)
    S = T + new + 8
    res = Generator(m, max_batch=1, max_seq=S, use_graphs=False, prefill_chunk=chunk, kv_dtype=kv_dtype)
    kv = HeadInferKV(cfg, 1, S, h_on=1, device=cuda, chunk_size=chunk, kv_dtype=kv_dtype)
    off = Generator(m, max_batch=1, max_seq=S, kv=kv)
    logits = []
    for gen in (res, off):
        gen.start(prompt, sp, seed=0)
        row = [gen._run["prefill_logits"].float().cpu()]
        gen.step(new - 1, record_latency=False)
        logits.append((gen.collect().tokens, row))
    (t_res, l_res), (t_off, l_off) = logits
    assert t_off == t_res
    for a, b in zip(l_off, l_res):
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 2e-2, rel
    if kv_dtype == "int8":
        assert kv.bytes_h2d > 0 and kv.host_k.dtype == torch.int8

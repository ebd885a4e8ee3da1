"""Pipeline runtime on the GPU: two gloo ranks share one device (P2P staged through host memory),
so stage compute, HIP graph capture/replay per (micro-batch, length bucket), the token ring
and the sampler run exactly as on a multi-GPU node — only the transport differs from RCCL.

Split must equal unsplit token-for-token: every layer runs the same kernels on the same
micro-batch shape whether it lives in one process or two.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from edgellm.engine import Generator, SamplingParams
from edgellm.models import build_model, tiny
from edgellm.parallel.partition import partition_model

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(arch, quant, first=0, last=None):
    from edgellm.quant import quantize_model
    cfg = tiny(arch, num_layers=4)
    model = build_model(cfg, dtype=torch.bfloat16, device="cuda:0", first=first, last=last, seed=7)
    if quant != "none":
        model = quantize_model(model, quant)
    return cfg, model


def _sampling(S, do_sample):
    return SamplingParams(max_new_tokens=S + 1, do_sample=do_sample, temperature=0.7, top_k=20, top_p=0.9,
                          repetition_penalty=1.1)


def _worker(rank, world, port, arch, quant, M, b, T, S, do_sample, q, lanes=1, headinfer_heads=None,
            prefill_chunk=4096, vocab_split=False):
    import edgellm  # noqa: F401
    from edgellm.parallel.pipeline import PipelineStage
    from datetime import timedelta
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # a rank that dies must not leave its peer blocked in a gloo recv for gloo's 30-min default
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    torch.cuda.set_device(0)
    cfg = tiny(arch, num_layers=4)
    bounds = partition_model(cfg, world, "uniform")
    _, model = _model(arch, quant, bounds[rank], bounds[rank + 1])
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)]
    shard = None
    if vocab_split:
        from edgellm.parallel.vocab_head import build_head_shard
        shard = build_head_shard(cfg, rank, world, model=model, seed=7, dtype=torch.bfloat16, device="cuda:0")
    st = PipelineStage(model, rank, world, b, M, max_seq=T + S + 4, lanes=lanes, headinfer_heads=headinfer_heads,
                       prefill_chunk=prefill_chunk, vocab_split=vocab_split, head_shard=shard)
    assert st.host_staged and st.use_graphs
    lag = world + 1 if vocab_split else world - 1
    n_ticks = (M + S * M) // lanes + lag
    res = st.run(prompts if rank == 0 else None, T, _sampling(S, do_sample), S, seed=5,
                 stats_window=(M // lanes + lag, n_ticks))
    assert st.vs == vocab_split
    assert res.stats["compute_ms_per_tick"] > 0 and 0 <= res.stats["bubble_frac"] <= 1
    if res.tokens is not None:
        q.put(res.tokens)
    dist.barrier()
    dist.destroy_process_group()


def _reference(arch, quant, M, b, T, S, do_sample, prefill_chunk=None, headinfer_heads=None):
    """Unsplit model, one micro-batch at a time.  With HeadInfer the reference runs the same
    offload path (HeadInferKV under the Generator): offloaded attention is the unfused
    RoPE-append + attention pair with a per-token-quantised o-projection input, so it is not
    bit-identical to the resident fused decode kernel and near-tied samples may differ from a
    resident run (that comparison is a tolerance test in tests/test_headinfer*.py)."""
    cfg, model = _model(arch, quant)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)]
    out = []
    kv = None
    if headinfer_heads is not None:
        from edgellm.offload import HeadInferKV
        kv = HeadInferKV(cfg, b, T + S + 4, headinfer_heads, model.device, chunk_size=min(T, prefill_chunk),
                         dtype=model.dtype)
    gen = Generator(model, max_batch=b, max_seq=T + S + 4, prefill_chunk=prefill_chunk, kv=kv)
    for m in range(M):
        out.extend(gen.generate(prompts[m].tolist(), _sampling(S, do_sample), seed=(5 + 7919 * m) & 0x7FFFFFFF).tokens)
    return out


@pytest.mark.parametrize("quant,lanes,world", [("none", 1, 2), ("w8a8", 1, 2), ("w8a8", 2, 2), ("w8a8", 2, 4)])
@pytest.mark.parametrize("do_sample", [False, True])
def test_pipeline_gpu_matches_unsplit(cuda, quant, lanes, world, do_sample):
    """lanes = 2: two micro-batches per tick on two HIP streams (own graph pools) per stage;
    world 4: one layer per stage, the driver's 4-way split shape."""
    _run(quant, lanes, world, do_sample)


@pytest.mark.parametrize("world", [2, 4])
def test_pipeline_gpu_headinfer_chunked(cuda, world):
    """Pipeline + HeadInfer on the device: 1 of 2 KV heads per layer offloaded to pinned host
    memory, prefill in 4-token chunks; tokens equal the unsplit model's on the same offload path."""
    _run("w8a8", 1, world, True, headinfer_heads=1, prefill_chunk=4)


@pytest.mark.parametrize("quant,lanes,world", [("none", 1, 2), ("w8a8", 2, 2), ("w8a8", 1, 4)])
@pytest.mark.parametrize("do_sample", [False, True])
def test_pipeline_gpu_vocab_split_matches_unsplit(cuda, quant, lanes, world, do_sample):
    """LM head split by vocabulary over the ranks (every rank its logits slice + the sampler's
    phase 1 on the GPU, rank 0 the merge kernel): tokens equal the unsplit model's."""
    _run(quant, lanes, world, do_sample, vocab_split=True)


def _run(quant, lanes, world, do_sample, headinfer_heads=None, prefill_chunk=4096, vocab_split=False):
    arch, b, T, S = "llama", 4, 9, 12
    M = (world + 1 if vocab_split else world) * lanes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, arch, quant, M, b, T, S, do_sample, q, lanes,
                                               headinfer_heads, prefill_chunk, vocab_split))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=150)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    ref = _reference(arch, quant, M, b, T, S, do_sample, prefill_chunk if headinfer_heads else None, headinfer_heads)
    bad = [i for i, (x, y) in enumerate(zip(got, ref)) if x != y]
    assert got == ref, f"rows {bad}: " + "; ".join(f"{got[i]} != {ref[i]}" for i in bad[:4])

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


def _worker(rank, world, port, arch, quant, M, b, T, S, do_sample, q, lanes=1):
    import edgellm  # noqa: F401
    from edgellm.parallel.pipeline import PipelineStage
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    cfg = tiny(arch, num_layers=4)
    bounds = partition_model(cfg, world, "uniform")
    _, model = _model(arch, quant, bounds[rank], bounds[rank + 1])
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)]
    st = PipelineStage(model, rank, world, b, M, max_seq=T + S + 4, lanes=lanes)
    assert st.host_staged and st.use_graphs
    res = st.run(prompts if rank == 0 else None, T, _sampling(S, do_sample), S, seed=5)
    if res.tokens is not None:
        q.put(res.tokens)
    dist.barrier()
    dist.destroy_process_group()


def _reference(arch, quant, M, b, T, S, do_sample):
    cfg, model = _model(arch, quant)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)]
    out = []
    gen = Generator(model, max_batch=b, max_seq=T + S + 4)
    for m in range(M):
        out.extend(gen.generate(prompts[m].tolist(), _sampling(S, do_sample), seed=(5 + 7919 * m) & 0x7FFFFFFF).tokens)
    return out


@pytest.mark.parametrize("quant,lanes", [("none", 1), ("w8a8", 1), ("w8a8", 2)])
@pytest.mark.parametrize("do_sample", [False, True])
def test_pipeline_gpu_matches_unsplit(cuda, quant, lanes, do_sample):
    """lanes = 2: two micro-batches per tick on two HIP streams (own graph pools) per stage."""
    arch, world, b, T, S = "llama", 2, 4, 9, 12
    M = world * lanes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, arch, quant, M, b, T, S, do_sample, q, lanes))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    assert got == _reference(arch, quant, M, b, T, S, do_sample)

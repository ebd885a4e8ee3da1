"""Pipeline runtime on CPU with the gloo backend (multi-process, world_size 2, 3, 4 and 8).

Every exchange goes through the same ``dist.P2POp`` / ``batch_isend_irecv`` code the RCCL run
uses; world 4 and 8 rehearse the driver's 4- and 8-GPU splits (8 layers: one or two per stage,
plus the head stage), with one and two lanes and with HeadInfer offload.

Checks the split model's tokens are identical to the unsplit model's (greedy and seeded
sampling) — the SURVEY §4 requirement "a split model's output is bit-identical (greedy) to the
unsplit model".
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from edgellm.engine import Generator, SamplingParams
from edgellm.models import build_model, tiny
from edgellm.parallel.partition import balanced_partition, partition_model, stage_costs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, arch, M, b, T, S, do_sample, q, headinfer_heads=None, lanes=1, n_layers=4,
            prefill_chunk=4096):
    import edgellm  # noqa: F401
    from edgellm.parallel.pipeline import PipelineStage
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    cfg = tiny(arch, num_layers=n_layers)
    bounds = partition_model(cfg, world, "uniform")
    model = build_model(cfg, dtype=torch.float32, first=bounds[rank], last=bounds[rank + 1], seed=7)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)]
    st = PipelineStage(model, rank, world, b, M, max_seq=T + S + 4, headinfer_heads=headinfer_heads, lanes=lanes,
                       prefill_chunk=prefill_chunk)
    sp = SamplingParams(max_new_tokens=S + 1, do_sample=do_sample, temperature=0.7, top_k=20, top_p=0.9,
                        repetition_penalty=1.1)
    n_ticks = (M + S * M) // lanes + world - 1
    res = st.run(prompts if rank == 0 else None, T, sp, S, seed=5, stats_window=(M // lanes + world - 1, n_ticks))
    assert res.stats["ticks"] > 0 and 0.0 <= res.stats["bubble_frac"] <= 1.0, res.stats
    if world > 1:
        assert res.stats["p2p_bytes_per_tick"] > 0, res.stats
    if res.tokens is not None:
        q.put(res.tokens)
    dist.barrier()
    dist.destroy_process_group()


def _reference(arch, M, b, T, S, do_sample, n_layers=4):
    cfg = tiny(arch, num_layers=n_layers)
    model = build_model(cfg, dtype=torch.float32, seed=7)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)]
    sp = SamplingParams(max_new_tokens=S + 1, do_sample=do_sample, temperature=0.7, top_k=20, top_p=0.9,
                        repetition_penalty=1.1)
    out = []
    gen = Generator(model, max_batch=b, max_seq=T + S + 4)
    for m in range(M):
        out.extend(gen.generate(prompts[m].tolist(), sp, seed=(5 + 7919 * m) & 0x7FFFFFFF).tokens)
    return out


@pytest.mark.parametrize("world,M,lanes", [(2, 2, 1), (2, 3, 1), (3, 3, 1), (2, 4, 2), (3, 6, 2)])
@pytest.mark.parametrize("do_sample", [False, True])
def test_pipeline_matches_unsplit(world, M, lanes, do_sample):
    """Split == unsplit token for token, also with 2 lanes (two micro-batches per tick)."""
    arch, b, T, S = "llama", 2, 5, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, arch, M, b, T, S, do_sample, q, None, lanes))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == _reference(arch, M, b, T, S, do_sample)


def _run_world(world, M, lanes, do_sample, headinfer_heads=None, n_layers=8, T=5, S=6, prefill_chunk=4096):
    arch, b = "llama", 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, arch, M, b, T, S, do_sample, q, headinfer_heads,
                                               lanes, n_layers, prefill_chunk))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    assert got == _reference(arch, M, b, T, S, do_sample, n_layers)


@pytest.mark.parametrize("world,M,lanes", [(4, 4, 1), (4, 8, 2), (8, 8, 1), (8, 16, 2)])
def test_pipeline_world_4_8_matches_unsplit(world, M, lanes):
    """The driver's 4- and 8-stage splits (8 layers: 2 or 1 per stage, head on the last),
    sampled decode, through the P2POp exchange: tokens equal the unsplit model's."""
    torch.set_num_threads(1)
    _run_world(world, M, lanes, True)


@pytest.mark.parametrize("world", [4, 8])
def test_pipeline_world_4_8_headinfer_chunked_prefill(world):
    """BASELINE config 4 rehearsal: every stage offloads 1 of 2 KV heads, prefill runs in
    3-token chunks across the stages; tokens equal the unsplit, fully resident model's."""
    torch.set_num_threads(1)
    _run_world(world, world, 1, True, headinfer_heads=1, T=7, prefill_chunk=3)


def test_pipeline_headinfer_rejects_lanes():
    cfg = tiny("llama", num_layers=2)
    model = build_model(cfg, dtype=torch.float32, seed=7)
    from edgellm.parallel.pipeline import PipelineStage
    with pytest.raises(AssertionError, match="one stream"):
        PipelineStage(model, 0, 1, 1, 2, max_seq=16, headinfer_heads=1, lanes=2)


def test_pipeline_with_headinfer_offload_matches_unsplit():
    """BASELINE config 'pipeline + HeadInfer': each stage keeps 1 of 2 KV heads on the device and
    offloads the other to (pinned) host memory; tokens equal the unsplit, fully resident model's."""
    world, M, arch, b, T, S = 2, 2, "llama", 2, 5, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, arch, M, b, T, S, True, q, 1)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == _reference(arch, M, b, T, S, True)


def _stall_worker(rank, world, port, marker):
    import time as _t
    import edgellm  # noqa: F401
    from edgellm.parallel.pipeline import PipelineStage
    from edgellm.parallel.watchdog import Watchdog
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = tiny("llama", num_layers=2)
    model = build_model(cfg, dtype=torch.float32, first=rank, last=rank + 1, seed=7)
    st = PipelineStage(model, rank, world, 1, 2, max_seq=32)
    def on_timeout(msg):
        with open(marker, "w") as f:
            f.write(f"{rank}|{msg}")
        os._exit(0)

    wd = Watchdog(timeout_s=1.5, on_timeout=on_timeout)

    def fault(t):  # rank 1 hangs at tick 3 (a dead peer); rank 0's watchdog must fire
        if rank == 1 and t == 3:
            wd.stop()           # a hung/dead process reports nothing itself
            _t.sleep(30)
            os._exit(0)

    prompts = [torch.randint(0, cfg.vocab_size, (1, 4)) for _ in range(2)]
    with wd:
        st.run(prompts if rank == 0 else None, 4, SamplingParams(max_new_tokens=8, do_sample=False), 6,
               watchdog=wd, fault=fault)


def test_watchdog_detects_stalled_peer(tmp_path):
    ctx = mp.get_context("spawn")
    marker = str(tmp_path / "fired")
    port = _free_port()
    procs = [ctx.Process(target=_stall_worker, args=(r, 2, port, marker)) for r in range(2)]
    for p in procs:
        p.start()
    procs[0].join(timeout=120)
    for p in procs:
        if p.is_alive():
            p.kill()
    rank, msg = open(marker).read().split("|", 1)
    assert rank == "0" and "no progress" in msg


def test_balanced_partition():
    costs = [1.0] * 32
    b = balanced_partition(costs, 8, head_cost=1.3)
    assert b[0] == 0 and b[-1] == 32 and len(b) == 9
    from edgellm.models import get_config
    cfg = get_config("llama-2-7b")
    for P in (1, 2, 4, 8):
        bounds = partition_model(cfg, P)
        c = stage_costs(cfg, bounds)
        assert max(c) <= min(c) + cfg.layer_bytes(1.0) + 2 * cfg.hidden_size * cfg.vocab_size
    assert partition_model(cfg, 4, explicit="9,8,8,7") == [0, 9, 17, 25, 32]
    # decode-time costs: the head + sampler is 0.6 of a layer, so 8 stages of 4 layers beat the
    # byte model's 4,4,4,4,4,4,5,3 (which puts 5 layers on one stage)
    assert partition_model(cfg, 8, head_cost_layers=0.6) == [0, 4, 8, 12, 16, 20, 24, 28, 32]
    assert max(stage_costs(cfg, partition_model(cfg, 8, head_cost_layers=0.6), head_cost_layers=0.6)) \
        < max(stage_costs(cfg, partition_model(cfg, 8), head_cost_layers=0.6))

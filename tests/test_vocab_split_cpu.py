"""LM head split by vocabulary over the pipeline's ranks (parallel/vocab_head.py), CPU / gloo.

* Sampler phase 1 over vocab shards + the merge draw exactly the unsplit sampler's token
  (greedy, full-vocab sampling, top-k + top-p, repetition penalty), for any shard count.
* Pipelines of 2 / 4 / 8 ranks (sub-layer bounds, 1 and 2 lanes, slack 1) with the head split over
  every rank give the unsplit model's tokens, greedy and sampled.
* The unit partitioner with the head spread over the stages models a max / mean stage cost of
  <= 1.04 at 8 stages and <= 1.02 at 4 (Llama-2-7B, bench context), where a whole head on the
  last stage models 1.11 / 1.05.
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from edgellm import ops
from edgellm.engine import SamplingParams
from edgellm.models import build_model, tiny
from edgellm.ops import _ref
from edgellm.parallel.vocab_head import build_head_shard, shard_bounds
from test_pipeline_cpu import _free_port, _reference

CFGS = [(0.7, 50, 0.9, 1.1, True), (1.0, 0, 1.0, 1.3, True), (0.5, 0, 1.0, 1.0, True),
        (0.7, 20, 1.0, 1.2, False), (0.8, 7, 0.5, 1.1, True), (0.7, 100, 0.95, 1.1, True)]


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_shard_sampler_equals_unsplit(cfg, P):
    T, k, p, pen, ds = cfg
    torch.manual_seed(0)
    B, V = 5, 1000
    logits = (torch.randn(B, V) * 3).bfloat16().float()      # bf16-valued scores: many exact ties
    seen = (torch.rand(B, V) < 0.1).to(torch.uint8)
    rng = torch.tensor([123, 9], dtype=torch.int32)
    ref = _ref.sample(logits, seen, T, k, p, pen, 123, 9, ds)
    b = shard_bounds(V, P, align=8)
    shards = [ops.sample_shard(logits[:, b[r]:b[r + 1]], seen[:, b[r]:b[r + 1]], T, k, p, pen, rng, b[r], V, ds)
              for r in range(P)]
    assert torch.equal(ops.sample_merge(shards, V, T, k, p, rng, ds), ref)


def test_shard_mode_and_bounds():
    assert ops.shard_mode(0.7, 50, 0.9, 32000) == 2
    assert ops.shard_mode(0.7, 0, 1.0, 32000) == 1
    assert ops.shard_mode(0.7, 50, 0.9, 32000, do_sample=False) == 0
    assert ops.shard_mode(0.7, 0, 0.9, 32000) == -1          # top-p without top-k: a full sort
    assert ops.shard_mode(0.7, 500, 1.0, 32000) == -1        # top-k beyond the candidate lists
    b = shard_bounds(32000, 8)
    assert b[0] == 0 and b[-1] == 32000 and all(x % 64 == 0 for x in b[:-1])
    assert max(b[r + 1] - b[r] for r in range(8)) - min(b[r + 1] - b[r] for r in range(8)) <= 64 * 8
    with pytest.raises(AssertionError):
        shard_bounds(100, 8)


def test_seen_mark_only_in_shard():
    seen = torch.zeros(3, 10, dtype=torch.uint8)
    seen[1, 4] = 1
    ops.seen_mark(seen, torch.tensor([25, 3, 19]), 20)      # shard [20, 30)
    assert seen[0, 5] == 1 and seen[1, 4] == 1 and seen.sum() == 2
    ops.seen_mark(seen, torch.tensor([25, 3, 19]), 20)      # idempotent
    assert seen.sum() == 2


def test_head_shard_matches_full_head():
    cfg = tiny("llama2", num_layers=2)
    full = build_model(cfg, dtype=torch.float32, seed=7)
    h = torch.randn(3, cfg.hidden_size)
    ref = torch.nn.functional.linear(h, full.lm_head.weight)
    parts = []
    for r in range(4):                         # from the random-init head (a rank without the head)
        sh = build_head_shard(cfg, r, 4, model=None, seed=7, dtype=torch.float32)
        parts.append(sh.logits(h))
    assert torch.allclose(torch.cat(parts, 1), ref)
    sh = build_head_shard(cfg, 3, 4, model=full, dtype=torch.float32)   # from a stage holding the head
    assert torch.equal(sh.proj.weight, full.lm_head.weight[sh.v0:sh.v1])


def _worker(rank, world, port, ubounds, M, b, T, S, slack, lanes, do_sample, q):
    import edgellm  # noqa: F401
    from edgellm.parallel.pipeline import PipelineStage
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    cfg = tiny("llama", num_layers=8)
    model = build_model(cfg, dtype=torch.float32, seed=7, units=(ubounds[rank], ubounds[rank + 1]))
    shard = build_head_shard(cfg, rank, world, model=model, seed=7, dtype=torch.float32)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)]
    st = PipelineStage(model, rank, world, b, M, max_seq=T + S + 4, lanes=lanes, slack=slack, vocab_split=True,
                       head_shard=shard)
    sp = SamplingParams(max_new_tokens=S + 1, do_sample=do_sample, temperature=0.7, top_k=20, top_p=0.9,
                        repetition_penalty=1.1)
    D = 1 + slack
    n_ticks = (M + S * M) // lanes + D * (world + 1)
    res = st.run(prompts if rank == 0 else None, T, sp, S, seed=5,
                 stats_window=(M // lanes + D * (world + 1), n_ticks))
    assert st.vs
    assert res.stats["ticks"] > 0, res.stats
    assert (res.tokens is not None) == (rank == 0)
    if res.tokens is not None:
        q.put(res.tokens)
    dist.barrier()
    dist.destroy_process_group()


def _run(world, ubounds, groups, slack=0, lanes=1, do_sample=True, T=5, S=6, b=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    M = groups * lanes
    procs = [ctx.Process(target=_worker, args=(r, world, port, ubounds, M, b, T, S, slack, lanes, do_sample, q))
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
    assert got == _reference("llama", M, b, T, S, do_sample, 8)


@pytest.mark.parametrize("do_sample", [True, False])
@pytest.mark.parametrize("world,ubounds", [(2, [0, 7, 16]), (4, [0, 3, 8, 13, 16]),
                                           (8, [0, 3, 5, 7, 8, 9, 12, 15, 16])])
def test_vocab_split_pipeline_matches_unsplit(world, ubounds, do_sample):
    """P + 1 micro-batch groups in flight (the token takes two more ticks to reach rank 0)."""
    torch.set_num_threads(1)
    _run(world, ubounds, world + 1, do_sample=do_sample)


def test_vocab_split_lanes_and_slack():
    torch.set_num_threads(1)
    _run(2, [0, 9, 16], 3, lanes=2)                    # two lanes, per-lane exchanges
    _run(2, [0, 9, 16], 6, slack=1)                     # every hop one tick behind: 2 (P + 1) groups


def test_vocab_split_needs_groups():
    cfg = tiny("llama", num_layers=2)
    from edgellm.parallel.pipeline import PipelineStage
    st = PipelineStage(build_model(cfg, dtype=torch.float32, seed=7), 0, 1, 1, 1, max_seq=16, vocab_split=True)
    assert not st.vs_req                                # one rank: nothing to split

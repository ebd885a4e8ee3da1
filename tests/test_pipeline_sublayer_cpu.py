"""Sub-layer stage boundaries and the slack schedule of the pipeline (CPU, gloo, worlds 2 / 4 / 8).

* A stage boundary may fall between a layer's attention half (norm1 + attention + o) and its MLP
  half (norm2 + MLP): the hand-off is the residual stream h2 = a + h, the same single tensor a
  whole-layer boundary hands over (``DecoderLM.from_units``).  Tokens equal the unsplit model's.
* ``slack=1``: a group reaches the next stage two ticks later, so each exchange completes one tick
  after it is posted — the hop runs beside a tick of compute — with 2P micro-batch groups in flight.
  Tokens are unchanged.
* The unit partitioner balances at least as well as whole layers, and its stage costs follow the
  cost model.
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from edgellm.models import build_model, tiny
from edgellm.models.decoder import DecoderLM
from test_pipeline_cpu import _free_port, _reference


def _worker(rank, world, port, ubounds, M, b, T, S, slack, q, lanes=1, quant="none"):
    import edgellm  # noqa: F401
    from edgellm.parallel.pipeline import PipelineStage
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    cfg = tiny("llama", num_layers=8)
    model = build_model(cfg, dtype=torch.float32, seed=7, units=(ubounds[rank], ubounds[rank + 1]))
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)]
    st = PipelineStage(model, rank, world, b, M, max_seq=T + S + 4, lanes=lanes, slack=slack)
    sp = SamplingParams(max_new_tokens=S + 1, do_sample=True, temperature=0.7, top_k=20, top_p=0.9,
                        repetition_penalty=1.1)
    D = 1 + slack
    n_ticks = (M + S * M) // lanes + D * (world - 1)
    res = st.run(prompts if rank == 0 else None, T, sp, S, seed=5,
                 stats_window=(M // lanes + D * (world - 1), n_ticks))
    assert res.stats["ticks"] > 0 and 0.0 <= res.stats["bubble_frac"] <= 1.0, res.stats
    if res.tokens is not None:
        q.put(res.tokens)
    dist.barrier()
    dist.destroy_process_group()


from edgellm.engine import SamplingParams  # noqa: E402


def _run(world, ubounds, M, slack, lanes=1, T=5, S=6, b=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ubounds, M, b, T, S, slack, q, lanes))
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
    assert got == _reference("llama", M, b, T, S, True, 8)


@pytest.mark.parametrize("world,ubounds", [(2, [0, 7, 16]), (4, [0, 3, 8, 13, 16]),
                                           (8, [0, 3, 5, 7, 8, 9, 12, 15, 16])])
def test_sublayer_bounds_match_unsplit(world, ubounds):
    """Stages cut mid-layer (odd unit bounds: the MLP half of a layer on the next stage)."""
    torch.set_num_threads(1)
    _run(world, ubounds, world, 0)


@pytest.mark.parametrize("world,ubounds", [(2, [0, 9, 16]), (4, [0, 3, 8, 13, 16])])
def test_slack_schedule_matches_unsplit(world, ubounds):
    """slack 1: 2 (P - 1) + 2 = 2P micro-batch groups in flight, every hop a tick behind."""
    torch.set_num_threads(1)
    _run(world, ubounds, 2 * world, 1)


def test_slack_needs_groups():
    cfg = tiny("llama", num_layers=2)
    from edgellm.parallel.pipeline import PipelineStage
    st = PipelineStage(build_model(cfg, dtype=torch.float32, seed=7), 0, 1, 1, 1, max_seq=16, slack=1)
    assert st.slack == 1                      # world 1: nothing to overlap, any M works


def test_half_layer_modules_and_weights():
    """A stage opening on an MLP half holds no attention (and no KV) for that layer; the halves of
    a split layer carry exactly the unsplit layer's parameters."""
    cfg = tiny("llama", num_layers=4)
    full = build_model(cfg, dtype=torch.float32, seed=3)
    a = build_model(cfg, dtype=torch.float32, seed=3, units=(0, 5))     # layers 0, 1 + attention of 2
    z = build_model(cfg, dtype=torch.float32, seed=3, units=(5, 8))     # MLP of 2, layer 3 + head
    assert a.has_embed and not a.has_head and z.has_head and not z.has_embed
    assert a.layers[-1].mlp is None and a.layers[-1].attn is not None
    assert z.layers[0].attn is None and z.layers[0].norm1 is None and z.kv_first == 3
    from edgellm.models.decoder import global_named_parameters
    ref = dict(global_named_parameters(full))
    got = {**dict(global_named_parameters(a)), **dict(global_named_parameters(z))}
    if cfg.tie_word_embeddings:                 # a head-only stage holds its own copy of the tied head
        assert torch.equal(got.pop("lm_head.weight"), ref["embed"])
    assert set(got) == set(ref)
    assert all(torch.equal(got[k], ref[k]) for k in ref)
    with pytest.raises(AssertionError):
        DecoderLM.from_units(tiny("phi", num_layers=2), 0, 1)       # parallel residual: whole layers only


def test_unit_partition_balance():
    from edgellm.models import get_config
    from edgellm.parallel.partition import partition_model, partition_units, unit_stage_costs
    cfg = get_config("llama-2-7b")
    for P in (2, 4, 8):
        ub = partition_units(cfg, P)
        assert ub[0] == 0 and ub[-1] == 2 * cfg.num_layers and all(x < y for x, y in zip(ub, ub[1:]))
        whole = [2 * x for x in partition_model(cfg, P, "balanced", head_cost_layers=0.52)]
        assert max(unit_stage_costs(cfg, ub)) <= max(unit_stage_costs(cfg, whole)) + 1e-6
    # a short context (small attention halves) is where the half-layer cut pays at 8 stages
    ub = partition_units(cfg, 8, ctx=16)
    c = unit_stage_costs(cfg, ub, ctx=16)
    w = unit_stage_costs(cfg, [2 * x for x in partition_model(cfg, 8, "balanced", head_cost_layers=0.52)], ctx=16)
    assert max(c) / (sum(c) / 8) < max(w) / (sum(w) / 8)

"""Pipeline serving engine (parallel/pp_engine.py) on CPU with gloo, 2 and 3 ranks.

The driver (rank 0) issues generate / confidence commands, the other ranks serve them from their
stage.  Ragged prompts (one right-padded prefill pass per micro-batch), EOS agreement and the
confidence metric through the pipeline are checked against the unsplit single-process engine:
greedy tokens identical, seeded sampling identical to the same micro-batches on lanes.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from edgellm.engine import Generator, SamplingParams
from edgellm.engine.generate import LaneGenerator
from edgellm.eval.metrics import confidence_score
from edgellm.models import build_model, tiny

PROMPTS = [[3, 14, 15, 92, 65, 35, 89], [7, 1], [22, 4, 9, 9, 31], [5], [8, 8, 2, 40]]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(arch):
    return tiny(arch, num_layers=6)


def _worker(rank, world, port, arch, sp_kw, eos, q, prompts=PROMPTS, vs=False):
    import edgellm  # noqa: F401
    from edgellm.parallel.partition import partition_model
    from edgellm.parallel.pp_engine import PipelineGenerator, serve_workers, stop_workers
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    cfg = _cfg(arch)
    bounds = partition_model(cfg, world, "uniform")
    model = build_model(cfg, dtype=torch.float32, first=bounds[rank], last=bounds[rank + 1], seed=7)
    shard = None
    if vs:                                       # LM head split by vocabulary over the ranks
        from edgellm.parallel.vocab_head import shard_from_last_stage
        shard = shard_from_last_stage(model, cfg, rank, world)
    eng = PipelineGenerator(model, rank, world, max_batch=6, max_seq=40, tag=3, vocab_split=vs, head_shard=shard)
    if rank == 0:
        sp = SamplingParams(**sp_kw)
        res = eng.generate(prompts, sp, seed=11, eos_token_id=eos)
        ticks = eng.last_ticks
        conf = eng.confidence([5, 9, 2, 7, 7, 1])
        try:                                     # rejected on the driver before any command goes out
            eng.generate([[1] * 39], sp, seed=11)
            raise RuntimeError("an oversized job must be rejected")
        except AssertionError:
            pass
        again = eng.generate(prompts[:2], sp, seed=11, eos_token_id=eos)     # engine reuse, fewer rows
        stop_workers(eng)
        assert eng.stage.vs == vs                # (the last run's sampling shards whenever vs)
        q.put((res.tokens, conf, again.tokens, eng.stage.M, eng.stage.b, ticks))
    else:
        n = serve_workers({3: eng})
        assert n == 3, n
    dist.barrier()
    dist.destroy_process_group()


def _run(world, arch, sp_kw, eos=None, prompts=PROMPTS, vs=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, arch, sp_kw, eos, q, prompts, vs)) for r in range(world)]
    for p in ps:
        p.start()
    out = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


GREEDY = dict(max_new_tokens=8, do_sample=False, repetition_penalty=1.1)
SAMPLED = dict(max_new_tokens=8, do_sample=True, temperature=0.7, top_k=20, top_p=0.9, repetition_penalty=1.1)


@pytest.mark.parametrize("vs", [False, True])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("arch", ["llama", "gpt_neox"])
def test_pp_engine_greedy_ragged_matches_unsplit(world, arch, vs):
    toks, conf, again, M, b, ticks = _run(world, arch, GREEDY, vs=vs)
    full = build_model(_cfg(arch), dtype=torch.float32, seed=7)
    sp = SamplingParams(**GREEDY)
    for p, t in zip(PROMPTS, toks):
        assert t == Generator(full, max_batch=1, max_seq=40).generate([p], sp).tokens[0]
    assert again == toks[:2]
    assert abs(conf - confidence_score(full, [5, 9, 2, 7, 7, 1])) < 1e-5


@pytest.mark.parametrize("vs", [False, True])
def test_pp_engine_sampling_matches_lanes(vs):
    """Seeded sampling: micro-batch m samples with seed + 7919 m, exactly as LaneGenerator's lane m
    (also with the vocab-split head: one more micro-batch group, the same draws)."""
    toks, _, _, M, b, _ = _run(2, "llama", SAMPLED, vs=vs)
    full = build_model(_cfg("llama"), dtype=torch.float32, seed=7)
    rows = PROMPTS + [PROMPTS[0]] * (M * b - len(PROMPTS))
    lg = LaneGenerator(full, lanes=M, max_batch=b, max_seq=40)
    lg.start(rows, SamplingParams(**SAMPLED), seed=11)
    lg.step(SAMPLED["max_new_tokens"] - 1, record_latency=False)
    ref = [r for res in lg.collect() for r in res.tokens]
    assert toks == ref[:len(PROMPTS)]


def test_pp_engine_eos_exit():
    """An EOS every row produces early ends the pipeline before max_new_tokens on every rank
    (one all-reduce per check period); outputs are trimmed at EOS like Generator's."""
    full = build_model(_cfg("llama"), dtype=torch.float32, seed=7)
    p0 = PROMPTS[0]
    prompts = [p0, p0[:6], p0, p0[:3], p0[:6]]          # ragged; greedy rows all start with token 269
    sp = SamplingParams(**dict(GREEDY, max_new_tokens=30))
    ref = Generator(full, max_batch=len(prompts), max_seq=40).generate(prompts, sp)
    eos = ref.tokens[0][0]
    assert all(eos in r for r in ref.tokens)
    toks, _, _, M, _, ticks = _run(2, "llama", dict(GREEDY, max_new_tokens=30), eos=eos, prompts=prompts)
    full_ticks = M + 29 * M + 2 - 1                   # every decode round + the pipeline fill
    assert ticks < full_ticks // 2, (ticks, full_ticks)
    want = Generator(full, max_batch=len(prompts), max_seq=40).generate(prompts, sp, eos_token_id=eos).tokens
    assert toks == want
    toks, _, _, M, _, ticks = _run(2, "llama", dict(GREEDY, max_new_tokens=30), eos=eos, prompts=prompts, vs=True)
    assert toks == want and ticks < (M + 29 * M + 4) // 2         # EOS agreement from rank 0

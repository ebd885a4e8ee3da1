"""Continuous batching over the RCCL pipeline engine on the GPU (parallel.pp_slots), world 1.

A spawned child (its own time limit) brings up a world-1 RCCL process group and drives a
``PipelineSlotDecoder`` directly: three requests admitted by one command (one ragged prefill),
decode rounds that replay HIP graphs captured per (micro-batch, KV bucket), a fourth request
admitted mid-decode, rows stopping on the device at their own budgets.  The greedy tokens must
equal the single-process ``Generator`` on the same weights, and graphs must have been captured.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

REQS = [([5, 9, 2, 44, 17, 3], 30), ([8, 1, 77], 7), ([12, 4, 9, 9, 31, 2, 8, 1, 66], 22)]
LATE = ([3, 3, 7, 100, 21], 12)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(port, q):
    import edgellm  # noqa: F401
    from edgellm.engine import SamplingParams
    from edgellm.models import build_model, tiny
    from edgellm.parallel.pipeline import init_distributed
    from edgellm.parallel.pp_engine import PipelineGenerator
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    init_distributed("nccl", timeout_s=120)
    dev = torch.device("cuda", 0)
    model = build_model(tiny("llama", num_layers=3), device=dev, seed=11)
    eng = PipelineGenerator(model, 0, 1, max_batch=4, max_seq=128)
    sp = SamplingParams(max_new_tokens=1, do_sample=False, repetition_penalty=1.1)
    dec = eng.slot_decoder(sp, seed=0, width=256)
    slots = dec.admit_batch([(ids, mx, None, f"r{i}") for i, (ids, mx) in enumerate(REQS)])
    done, order = {}, []
    rounds = 0
    while dec.busy() or "late" not in done:
        if rounds == 3:
            dec.admit(LATE[0], LATE[1], None, "late")
        dec.step(4)
        rounds += 1
        for tag, res in dec.poll():
            done[tag] = res.tokens[0]
            order.append(tag)
        assert rounds < 200
    q.put(dict(tokens=done, order=order, slots=slots, graphs=len(dec.sess._graphs)))
    dist.destroy_process_group()


def test_pp_slots_rccl_world1_graphs(cuda):
    import torch.multiprocessing as mp
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, tiny
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    try:
        rec = q.get(timeout=150)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
            p.join()
    assert rec["graphs"] >= 1, rec
    # the 7-token request ends before the 30-token one it was admitted with
    assert rec["order"].index("r1") < rec["order"].index("r0"), rec["order"]
    model = build_model(tiny("llama", num_layers=3), device=cuda, seed=11)
    gen = Generator(model, max_batch=1, max_seq=128)
    for i, (ids, mx) in enumerate(REQS + [LATE]):
        tag = f"r{i}" if i < len(REQS) else "late"
        want = gen.generate([ids], SamplingParams(max_new_tokens=mx, do_sample=False, repetition_penalty=1.1))
        assert rec["tokens"][tag] == want.tokens[0], tag

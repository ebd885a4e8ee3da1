"""Serving / comm layer on CPU: TimeService + REST compatibility with the reference demo
(Code/gRPC/*), and the BASELINE.json CPU config — a GPT-2 2-stage layer split over localhost
gRPC — checked token-for-token against the single-process engine, with injected drops."""
import json
import re

import pytest
import torch

from edgellm.engine import Generator, SamplingParams
from edgellm.models import build_model, tiny
from edgellm.serve import wire
from edgellm.serve.stage_service import (EdgePipeline, FaultInjector, RemoteStage, StageForward, StageServer,
                                         decode_tensor, encode_tensor, serve_stage)
from edgellm.serve.time_service import (decode_time_response, encode_time_response, get_current_time, make_server)

TIME_RE = re.compile(r"^\d{4}-\d{2}-\d{2} \d{2}:\d{2}:\d{2}$")


def test_time_response_wire_format():
    # protoc encoding of TimeResponse{current_time="2025-02-24 13:24:31"}: tag 0x0A, len 19, utf-8
    s = "2025-02-24 13:24:31"
    enc = encode_time_response(s)
    assert enc == b"\x0a\x13" + s.encode()
    assert decode_time_response(enc) == s


def test_time_service_roundtrip():
    server = make_server(port=0, host="127.0.0.1")
    try:
        t = get_current_time(f"127.0.0.1:{server.port}", timeout=5)
        assert TIME_RE.match(t), t
    finally:
        server.stop(0)


def test_time_service_unreachable_raises_after_retries():
    with pytest.raises(RuntimeError):
        get_current_time("127.0.0.1:1", timeout=0.2, retries=1, backoff=0.01)


def test_rest_time_endpoint():
    from fastapi.testclient import TestClient
    from edgellm.serve.rest import make_app
    c = TestClient(make_app())
    r = c.get("/")
    assert r.status_code == 200 and set(r.json()) == {"current_time"} and TIME_RE.match(r.json()["current_time"])
    assert c.get("/health").json()["status"] == "ok"


def test_tensor_codec_roundtrip():
    for t in (torch.randn(3, 5).bfloat16(), torch.randn(2, 2), torch.arange(7)):
        u = decode_tensor(encode_tensor(t))
        assert u.dtype == t.dtype and torch.equal(u, t)
    m = StageForward(7, 3, 1, torch.randn(2, 4).bfloat16(), 11, SamplingParams(temperature=0.5, top_k=30), 99,
                     torch.tensor([[1, 2]]))
    d = StageForward.decode(m.encode())
    assert (d.seq_id, d.step, d.kind, d.start_pos, d.seed) == (7, 3, 1, 11, 99)
    assert d.sampling.top_k == 30 and abs(d.sampling.temperature - 0.5) < 1e-7
    assert torch.equal(d.hidden, m.hidden)
    assert wire.unpack_varints(wire.field_packed_varints(1, [1, 300, 70000])[2:]) == [1, 300, 70000]


@pytest.mark.parametrize("do_sample", [False, True])
@pytest.mark.parametrize("faults", [None, "drops"])
def test_gpt2_two_stage_grpc_matches_single_process(do_sample, faults):
    cfg = tiny("gpt2", num_layers=4)
    full = build_model(cfg, dtype=torch.float32, seed=11)
    s0 = build_model(cfg, dtype=torch.float32, first=0, last=2, seed=11)
    s1 = build_model(cfg, dtype=torch.float32, first=2, last=4, seed=11)
    stage = StageServer(s1, max_seq=64)
    server = serve_stage(stage, port=0)
    try:
        fi = FaultInjector(drop_prob=0.3, seed=1, drop_first_n=1) if faults else None
        remote = RemoteStage(f"127.0.0.1:{server.port}", timeout=10, retries=8, backoff=0.001, faults=fi)
        pipe = EdgePipeline(s0, [remote], max_seq=64)
        prompts = [[5, 6, 7, 8], [9, 10, 11, 12]]
        sp = SamplingParams(max_new_tokens=8, do_sample=do_sample, temperature=0.7, top_k=50, top_p=0.9,
                            repetition_penalty=1.1)
        got = pipe.generate(prompts, sp, seed=3)
        ref = Generator(full, max_batch=2, max_seq=64).generate(prompts, sp, seed=3)
        assert got.tokens == ref.tokens
        if faults:
            assert fi.dropped > 0 and remote.retried >= fi.dropped
        remote.close()
    finally:
        server.stop(0)


def test_serving_engine_batches_concurrent_requests(tmp_path):
    import threading
    from fastapi.testclient import TestClient
    from edgellm.serve.rest import make_app
    from edgellm.serve.server import ServingEngine
    from edgellm.utils.tokenizer import ByteTokenizer
    cfg = tiny("llama")
    m = build_model(cfg, dtype=torch.float32, seed=2)
    mpath = tmp_path / "serve_metrics.jsonl"
    eng = ServingEngine(Generator(m, max_batch=4, max_seq=128), ByteTokenizer(cfg.vocab_size), max_batch=4,
                        batch_wait_s=0.05, metrics_path=str(mpath), continuous=False)
    try:
        sp = SamplingParams(max_new_tokens=5, do_sample=False)
        futs = [eng.submit([1, 2, 3 + i], sp) for i in range(4)]
        outs = [f.result(timeout=60) for f in futs]
        assert all(len(o["tokens"]) == 5 for o in outs)
        assert eng.metrics()["requests"] == 4 and eng.metrics()["batches"] <= 2
        # batched results equal the single-request results
        alone = Generator(m, max_batch=1, max_seq=128).generate([[1, 2, 4]], sp)
        assert outs[1]["tokens"] == alone.tokens[0]
        c = TestClient(make_app(eng))
        r = c.post("/generate", json={"prompt": "hello", "max_new_tokens": 3, "do_sample": False})
        assert r.status_code == 200 and len(r.json()["tokens"]) == 3
        assert c.get("/metrics").json()["requests"] == 5
        recs = [json.loads(l) for l in mpath.read_text().splitlines()]     # one JSONL record per batch
        assert len(recs) == eng.metrics()["batches"] and sum(r["batch_size"] for r in recs) == 5
        assert all(r["event"] == "batch" and r["ttft_ms"] > 0 and r["generated_tokens"] > 0 for r in recs)
    finally:
        eng.close()


def test_serving_engine_static_close_serves_queued():
    """close() right after submits: the static loop still answers every queued request."""
    from edgellm.serve.server import ServingEngine
    from edgellm.utils.tokenizer import ByteTokenizer
    cfg = tiny("llama")
    m = build_model(cfg, dtype=torch.float32, seed=2)
    eng = ServingEngine(Generator(m, max_batch=2, max_seq=64), ByteTokenizer(cfg.vocab_size), max_batch=2,
                        batch_wait_s=0.0, continuous=False)
    sp = SamplingParams(max_new_tokens=3, do_sample=False)
    futs = [eng.submit([1, 2, 3 + i], sp) for i in range(5)]
    eng.q.put(None)                              # the close() sentinel behind the requests
    outs = [f.result(timeout=60) for f in futs]
    eng.close()
    assert all(len(o["tokens"]) == 3 for o in outs) and eng.metrics()["requests"] == 5


def test_serving_engine_continuous_batching(tmp_path):
    """Iteration-level batching: requests of different lengths / budgets arriving while others
    decode are admitted into free slots between steps, finished slots are reused at once, and every
    greedy result equals the request run alone."""
    import time as _time
    from edgellm.serve.server import ServingEngine
    from edgellm.utils.tokenizer import ByteTokenizer
    cfg = tiny("llama")
    m = build_model(cfg, dtype=torch.float32, seed=2)
    eng = ServingEngine(Generator(m, max_batch=3, max_seq=128), ByteTokenizer(cfg.vocab_size), steps_per_poll=2,
                        metrics_path=str(tmp_path / "m.jsonl"))
    assert eng.continuous
    reqs = [([1, 2, 3], 9), ([5, 6, 7, 8, 9, 10], 4), ([11], 12), ([4, 4, 2, 7], 6), ([9, 8], 3), ([3] * 20, 7)]
    try:
        futs = []
        for i, (ids, n) in enumerate(reqs):
            futs.append(eng.submit(ids, SamplingParams(max_new_tokens=n, do_sample=False, repetition_penalty=1.1)))
            if i == 2:
                _time.sleep(0.05)             # the rest arrive while the first three decode
        outs = [f.result(timeout=120) for f in futs]
        for (ids, n), o in zip(reqs, outs):
            sp = SamplingParams(max_new_tokens=n, do_sample=False, repetition_penalty=1.1)
            assert o["tokens"] == Generator(m, max_batch=1, max_seq=128).generate([ids], sp).tokens[0]
        st = eng.metrics()
        assert st["requests"] == 6 and st["sessions"] == 1 and st["max_concurrent"] == 3
        # 6 requests, 41 tokens, 3 slots: far fewer steps than running them one after another
        assert st["decode_steps"] < sum(n - 1 for _, n in reqs)
        # a sampling configuration change opens a new session once the running one drains
        o = eng.submit([1, 2], SamplingParams(max_new_tokens=5, temperature=0.8, top_k=10)).result(timeout=60)
        assert len(o["tokens"]) == 5 and eng.metrics()["sessions"] == 2
    finally:
        eng.close()


def test_serving_engine_continuous_rejects_and_budgets():
    """Continuous mode fails requests it can never admit (empty prompt, prompt + budget beyond the
    cache, a budget wider than the session) at once and keeps serving the rest; a max_new_tokens=1
    request admitted beside live slots returns exactly one token; ``max_batch`` caps the slots."""
    from edgellm.serve.server import ServingEngine
    from edgellm.utils.tokenizer import ByteTokenizer
    cfg = tiny("llama")
    m = build_model(cfg, dtype=torch.float32, seed=2)
    eng = ServingEngine(Generator(m, max_batch=4, max_seq=64), ByteTokenizer(cfg.vocab_size), max_batch=2,
                        steps_per_poll=1)
    try:
        sp = SamplingParams(max_new_tokens=6, do_sample=False)
        bad = [eng.submit([], sp), eng.submit([1] * 60, sp),
               eng.submit([1, 2], SamplingParams(max_new_tokens=4096, do_sample=False))]
        for f in bad:
            with pytest.raises(ValueError):
                f.result(timeout=10)
        long = eng.submit([1, 2, 3], SamplingParams(max_new_tokens=12, do_sample=False))
        one = eng.submit([4, 5], SamplingParams(max_new_tokens=1, do_sample=False))
        ok = eng.submit([7, 8, 9], sp)
        assert len(one.result(timeout=60)["tokens"]) == 1
        assert len(long.result(timeout=60)["tokens"]) == 12 and len(ok.result(timeout=60)["tokens"]) == 6
        alone = Generator(m, max_batch=1, max_seq=64).generate([[4, 5]], SamplingParams(max_new_tokens=1,
                                                                                        do_sample=False))
        assert one.result()["tokens"] == alone.tokens[0]
        st = eng.metrics()
        assert st["errors"] == 3 and st["requests"] == 3 and st["max_concurrent"] <= 2
    finally:
        eng.close()


def test_stage_server_replays_retried_step():
    cfg = tiny("gpt2", num_layers=2)
    s1 = build_model(cfg, dtype=torch.float32, first=1, last=2, seed=1)
    st = StageServer(s1, max_seq=32)
    h = torch.randn(3, cfg.hidden_size)
    sp = SamplingParams(temperature=0.7, top_k=5)
    m = StageForward(1, 0, 0, h, 0, sp, 5, torch.tensor([[1, 2, 3]]))
    a = st.forward(m)
    b = st.forward(m)          # same (seq, step): served from the replay cache
    assert a == b and st.replays == 1


def test_client_cli_prints_remote_time(capsys):
    from edgellm.cli.client import main
    server = make_server(port=0, host="127.0.0.1")
    try:
        t = main(["--address", f"127.0.0.1:{server.port}", "--timeout", "5"])
        assert TIME_RE.match(t) and f"Current Time from 127.0.0.1:{server.port}: {t}" in capsys.readouterr().out
    finally:
        server.stop(0)


def test_serve_cli_stage_and_engine():
    """cli.serve builds a stage server that an EdgePipeline drives, and an engine-backed REST app."""
    from fastapi.testclient import TestClient
    from edgellm.cli.serve import build, parse
    from edgellm.models.registry import load_model
    server, port, app, engine = build(parse(["--model", "tiny:gpt2", "--stage", "1:2", "--grpc-port", "0",
                                             "--no-rest", "--precision", "fp32", "--device", "cpu"]))
    try:
        first, _, _ = load_model("tiny:gpt2", "fp32", "none", "cpu", first=0, last=1)
        full, _, _ = load_model("tiny:gpt2", "fp32", "none", "cpu")
        pipe = EdgePipeline(first, [RemoteStage(f"127.0.0.1:{port}", timeout=10)], max_seq=64)
        sp = SamplingParams(max_new_tokens=5, do_sample=False)
        assert pipe.generate([[3, 4, 5]], sp).tokens == Generator(full, max_batch=1, max_seq=64).generate([[3, 4, 5]], sp).tokens
        assert get_current_time(f"127.0.0.1:{port}", timeout=5)       # TimeService rides along
    finally:
        server.stop(0)
    server, port, app, engine = build(parse(["--model", "tiny:llama", "--grpc-port", "0", "--precision", "fp32",
                                             "--device", "cpu", "--max-seq", "128"]))
    try:
        r = TestClient(app).post("/generate", json={"prompt_ids": [1, 2, 3], "max_new_tokens": 4, "do_sample": False})
        assert r.status_code == 200 and len(r.json()["tokens"]) == 4
    finally:
        engine.close()
        server.stop(0)

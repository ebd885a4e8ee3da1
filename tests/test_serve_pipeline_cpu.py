"""Serving over the multi-process pipeline (SURVEY §2.4 request concurrency; reference:
Code/gRPC/server.py:14 thread-pool server).  Under torchrun (2 ranks, gloo on CPU) rank 0's REST
engine drives the PipelineGenerator: concurrent POST /generate requests are batched into the
pipeline's micro-batches, and every answer equals the single-process engine's."""
import json
import os
import subprocess
import sys

import pytest
import torch

from test_pp_cli_cpu import ROOT, _free_port


def test_rest_generate_over_pipeline_matches_single_process(tmp_path):
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models.registry import load_model
    out = tmp_path / "served.json"
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests"), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "helpers",
                                                                         "pp_serve_worker.py"), str(out), "tiny:llama"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    got = json.loads(out.read_text())
    model, _, _ = load_model("tiny:llama", "fp32", "none", "cpu")
    gen = Generator(model, max_batch=1, max_seq=128)
    for req, toks in zip(got["requests"], got["tokens"]):
        sp = SamplingParams(max_new_tokens=req["max_new_tokens"], do_sample=False, temperature=0.7, top_k=50,
                            top_p=0.9, repetition_penalty=1.1)
        assert toks == gen.generate([req["prompt_ids"]], sp).tokens[0], req
    # continuous batching (the default): sessions of slots, no static batches
    assert got["metrics"]["requests"] == 6 and got["metrics"]["sessions"] >= 1 and got["metrics"]["batches"] == 0


def test_continuous_batching_over_pipeline(tmp_path):
    """Continuous batching over a 2-rank pipeline (parallel.pp_slots): a short request submitted
    while a long one decodes is admitted into a free row at the next command boundary and
    completes FIRST; both answers equal the single-process Generator's (greedy)."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models.registry import load_model
    out = tmp_path / "slots.json"
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests"), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "helpers", "pp_slots_worker.py"), str(out), "tiny:llama"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    got = json.loads(out.read_text())
    assert got["order"] == ["short", "long"], got
    assert got["steps_at_submit"] >= 4
    model, _, _ = load_model("tiny:llama", "fp32", "none", "cpu")
    gen = Generator(model, max_batch=1, max_seq=128)
    for key in ("long", "short"):
        ids, n, toks = got[key]
        sp = SamplingParams(max_new_tokens=n, do_sample=False, temperature=0.7, top_k=50, top_p=0.9,
                            repetition_penalty=1.1)
        assert toks == gen.generate([ids], sp).tokens[0], key
    assert got["metrics"]["max_concurrent"] == 2 and got["metrics"]["requests"] == 2


def test_serve_cli_torchrun_shutdown_releases_every_rank(tmp_path):
    """``torchrun -m edgellm.cli.serve`` (2 ranks, gloo): rank 0 serves REST over the pipeline; a
    SIGINT to rank 0 shuts uvicorn down, the engine drains, the worker rank is released
    (stop_workers from the app's shutdown) and the whole job exits 0 — no rank left blocked in
    the next command broadcast."""
    import signal
    import time
    import urllib.request
    import psutil
    rest, grpc_port = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", EDGELLM_PG_TIMEOUT_S="120")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "-m", "edgellm.cli.serve", "--model", "tiny:llama",
           "--device", "cpu", "--precision", "fp32", "--max-seq", "128", "--max-batch", "4",
           "--rest-port", str(rest), "--grpc-port", str(grpc_port), "--host", "127.0.0.1"]
    log = open(tmp_path / "serve.log", "w")
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT)
    try:
        url = f"http://127.0.0.1:{rest}"
        t0 = time.time()
        while True:
            assert p.poll() is None, open(tmp_path / "serve.log").read()[-3000:]
            try:
                urllib.request.urlopen(url + "/health", timeout=1).read()
                break
            except OSError:
                assert time.time() - t0 < 240, "server did not come up"
                time.sleep(0.5)
        body = json.dumps({"prompt_ids": [3, 4, 5], "max_new_tokens": 4, "do_sample": False}).encode()
        req = urllib.request.Request(url + "/generate", data=body, headers={"Content-Type": "application/json"})
        out = json.loads(urllib.request.urlopen(req, timeout=120).read())
        assert len(out["tokens"]) == 4
        rank0 = [c for c in psutil.Process(p.pid).children(recursive=True)
                 if c.environ().get("RANK") == "0" and c.environ().get("LOCAL_RANK") == "0"]
        assert len(rank0) == 1
        rank0[0].send_signal(signal.SIGINT)
        rc = p.wait(timeout=180)
    finally:
        if p.poll() is None:
            p.kill()
    assert rc == 0, open(tmp_path / "serve.log").read()[-3000:]


@pytest.mark.parametrize("vs", ["off", "on"])
def test_continuous_batching_4_ranks_staggered(tmp_path, vs):
    """16 staggered greedy requests over a 4-rank pipeline (parallel.pp_slots): queued requests
    are admitted together (one ragged prefill per command), every row stops on the device at its
    own token budget, a short request submitted while long ones decode finishes before all of
    them, and every answer equals the single-process Generator's.  ``vs`` on: the slots sample
    with the vocabulary-split head (every rank's logits slice + phase 1, rank 0 merges)."""
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models.registry import load_model
    out = tmp_path / "load.json"
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests"), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "helpers", "pp_slots_load_worker.py"), str(out), "tiny:llama", vs]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-4000:]
    got = json.loads(out.read_text())
    order = got["order"]
    assert sorted(order) == sorted(k for k, _, _ in got["requests"])
    assert order.index("short") < min(order.index(k) for k, _, mx in got["requests"] if mx >= 20), order
    model, _, _ = load_model("tiny:llama", "fp32", "none", "cpu")
    gen = Generator(model, max_batch=1, max_seq=128)
    for key, ids, mx in got["requests"]:
        sp = SamplingParams(max_new_tokens=mx, do_sample=False, temperature=0.7, top_k=50, top_p=0.9,
                            repetition_penalty=1.1)
        assert got["tokens"][key] == gen.generate([ids], sp).tokens[0], key
    m = got["metrics"]
    assert m["requests"] == 16 and m["max_concurrent"] >= 8
    assert got["vs_session"] == (vs == "on")

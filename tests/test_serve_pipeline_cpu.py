"""Serving over the multi-process pipeline (SURVEY §2.4 request concurrency; reference:
Code/gRPC/server.py:14 thread-pool server).  Under torchrun (2 ranks, gloo on CPU) rank 0's REST
engine drives the PipelineGenerator: concurrent POST /generate requests are batched into the
pipeline's micro-batches, and every answer equals the single-process engine's."""
import json
import os
import subprocess
import sys

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
    assert got["metrics"]["requests"] == 6 and got["metrics"]["batches"] >= 1

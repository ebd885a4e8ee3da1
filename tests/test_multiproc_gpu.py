"""The torchrun CLI paths on the GPU, rehearsed on one device: gloo ranks share cuda:0
(EDGELLM_DIST_BACKEND=gloo; pipeline P2P staged through pinned host memory), so the stage
compute, graph capture, command broadcasts and result delivery run exactly as under RCCL on a
multi-GPU node — only the transport differs.

* REST serving over a 2-stage pipeline (cli/serve.py ``build_pipeline_engine``): POST /generate
  answers equal the single-process Generator's, request by request (batch 1, greedy).
* The ensemble on disjoint rank groups (cli/combine.py, ``agents[].gpus``): 4 ranks, 2 agents x 2
  stages, majority vote — the answers equal the single-process GPU run of the same YAML, whose
  agents share the device through ``co_generate``.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from test_cli_cpu import _tiny_yaml
from test_pp_cli_cpu import ROOT, _free_port, _rows

pytestmark = pytest.mark.gpu


def _env():
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests"), OMP_NUM_THREADS="1",
               EDGELLM_DIST_BACKEND="gloo", EDGELLM_PG_TIMEOUT_S="120")
    env.pop("WORLD_SIZE", None)
    return env


def _torchrun(n, args, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), *args]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:]
    return r.stdout


def test_rest_generate_over_gpu_pipeline(cuda, tmp_path):
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models.registry import load_model
    out = tmp_path / "served.json"
    _torchrun(2, [os.path.join(ROOT, "tests", "helpers", "pp_serve_worker.py"), str(out), "tiny:llama", "cuda",
                  "bf16", "1", "seq"])
    got = json.loads(out.read_text())
    model, _, _ = load_model("tiny:llama", "bf16", "none", cuda)
    gen = Generator(model, max_batch=1, max_seq=128)
    for req, toks in zip(got["requests"], got["tokens"]):
        assert isinstance(toks, list) and len(toks) == req["max_new_tokens"], toks
        sp = SamplingParams(max_new_tokens=req["max_new_tokens"], do_sample=False, temperature=0.7, top_k=50,
                            top_p=0.9, repetition_penalty=1.1)
        assert toks == gen.generate([req["prompt_ids"]], sp).tokens[0], req
    assert got["metrics"]["requests"] == 6


def test_combine_agent_groups_on_gpu_match_single_process(cuda, tmp_path):
    from edgellm.cli import combine
    cfg = _tiny_yaml(tmp_path, """
merge: vote
agents:
  - {name: qa_llama, model: "tiny:llama", precision: bf16, gpus: [0, 1]}
  - {name: qa_neox, model: "tiny:gpt_neox", precision: bf16, gpus: [2, 3]}
""")
    args = ["--config", cfg, "--devices", "cuda:0", "--num_samples", "2", "--max_seq", "512"]
    single = tmp_path / "single.jsonl"
    combine.main(args + ["--metrics_jsonl", str(single)])
    grouped = tmp_path / "grouped.jsonl"
    log = _torchrun(4, ["-m", "edgellm.cli.combine", *args, "--metrics_jsonl", str(grouped)], timeout=300)
    assert "pipelined over 2 ranks [0, 1]" in log and "pipelined over 2 ranks [2, 3]" in log
    a, b = _rows(single), _rows(grouped)
    assert len(a) == len(b) == 2
    for x, y in zip(a, b):
        assert x["answers"] == y["answers"] and x["final"] == y["final"]

"""Multi-process ensemble on disjoint rank groups (BASELINE config 5 shape, CPU gloo).

* Under torchrun, ``agents[].gpus`` is each agent's rank group (one ``dist.new_group`` per agent):
  4 ranks, 2 QA agents x 2 pipeline stages each, majority-vote merge.  Both agents decode with ONE
  driver command and on disjoint ranks, so at the same time; the answers equal the single-process
  run of the same YAML (the reference runs its agents one after another,
  Code/Base Models/combine_model_fp_updated.py:194-200).
* ``run_agents`` dispatches on the engine's capability: a pipeline engine on a CUDA device is
  never handed to ``co_generate`` (which drives a plain Generator's internals).
"""
import json
import os
import subprocess
import sys

import torch

from test_cli_cpu import _tiny_yaml
from test_pp_cli_cpu import ROOT, _free_port, _rows


def test_pipeline_agents_never_reach_co_generate(monkeypatch):
    from edgellm.engine import GenerationResult, SamplingParams
    from edgellm.orchestrator import ensemble
    from edgellm.parallel import pp_engine
    from edgellm.utils.tokenizer import ByteTokenizer

    class FakeCudaPipeline(pp_engine.PipelineGenerator):
        def __init__(self, tag):                  # no stage, no process group: a driver-side shell
            self.tag, self.device, self.max_seq = tag, torch.device("cuda", 0), 64

    calls = []

    def fake_concurrent(jobs, stop_at_eos=True):
        calls.append([j[0].tag for j in jobs])
        return [GenerationResult([[65 + j[0].tag] * 3 for _ in j[1]], [len(p) for p in j[1]], 1.0, 0.1, 0.9)
                for j in jobs]

    def boom(*a, **k):
        raise AssertionError("co_generate must not drive a pipeline engine")

    monkeypatch.setattr(pp_engine, "generate_concurrent", fake_concurrent)
    monkeypatch.setattr(ensemble, "co_generate", boom)
    tok = ByteTokenizer(300)
    agents = [ensemble.Agent(f"a{i}", FakeCudaPipeline(i), tok, SamplingParams(max_new_tokens=3)) for i in range(3)]
    outs = ensemble.run_agents(agents, [["q1", "q2"]] * 3, [0, 1, 2], legacy_decode=False)
    assert calls == [[0, 1, 2]]                  # one concurrent command for every pipeline agent
    assert [o[0] for o in outs] == [[tok.decode([65 + i] * 3)] * 2 for i in range(3)]
    calls.clear()
    ensemble.run_agents(agents, [["q"]] * 3, [0, 1, 2], concurrent=False)
    assert calls == [[0], [1], [2]]              # --serial: one command per agent, in order


def test_combine_torchrun_agent_groups_match_single_process(tmp_path):
    extra = """
merge: vote
agents:
  - {name: qa_llama, model: "tiny:llama", precision: fp32, gpus: [0, 1]}
  - {name: qa_neox, model: "tiny:gpt_neox", precision: fp32, gpus: [2, 3]}
"""
    from edgellm.cli import combine
    cfg = _tiny_yaml(tmp_path, extra)
    args = ["--config", cfg, "--devices", "cpu", "--num_samples", "2", "--max_seq", "512"]
    single = tmp_path / "single.jsonl"
    combine.main(args + ["--metrics_jsonl", str(single)])
    grouped = tmp_path / "grouped.jsonl"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "-m", "edgellm.cli.combine", *args,
           "--metrics_jsonl", str(grouped)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "pipelined over 2 ranks [0, 1]" in r.stdout and "pipelined over 2 ranks [2, 3]" in r.stdout
    a, b = _rows(single), _rows(grouped)
    assert len(a) == len(b) == 2
    for x, y in zip(a, b):
        assert x["answers"] == y["answers"] and x["final"] == y["final"]

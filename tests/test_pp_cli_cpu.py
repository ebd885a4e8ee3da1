"""The combine CLI under torchrun (2 ranks, gloo on CPU): every agent's model runs as a pipeline
(parallel/pp_engine.py) instead of the eager SplitLM — QA agents, the refiner and the
confidence metric.  Answers, refined outputs and every metric equal the single-process run
(batch 1: micro-batch 0, row 0 samples with the same seed as the unsplit engine)."""
import json
import os
import socket
import subprocess
import sys

from test_cli_cpu import _tiny_yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def test_combine_torchrun_pipeline_matches_single_process(tmp_path):
    from edgellm.cli import combine
    cfg = _tiny_yaml(tmp_path)
    args = ["--config", cfg, "--devices", "cpu", "--num_samples", "2", "--max_seq", "1024", "--merge", "refine"]
    single = tmp_path / "single.jsonl"
    combine.main(args + ["--metrics_jsonl", str(single)])
    piped = tmp_path / "piped.jsonl"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "-m", "edgellm.cli.combine", *args,
           "--metrics_jsonl", str(piped)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "pipelined over 2 ranks" in r.stdout
    a, b = _rows(single), _rows(piped)
    assert len(a) == len(b) == 2
    for x, y in zip(a, b):
        assert x["answers"] == y["answers"] and x["final"] == y["final"]
        for k in ("rouge1", "rouge2", "rougeL", "bleu", "cosine", "bertscore"):
            assert x[k] == y[k], k
        assert abs(x["confidence"] - y["confidence"]) < 1e-4

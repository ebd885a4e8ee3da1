"""bench.py contract on CPU: single-process and torchrun (gloo, 2 ranks) legs print one JSON
line with the required fields (the driver runs the same script on MI355X with RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


COMMON = ["--device", "cpu", "--model", "tiny:llama", "--micro-batch", "2", "--steps", "3", "--warmup", "1",
          "--prompt-len", "6"]


@pytest.mark.parametrize("lanes", [1, 2])
def test_bench_single_cpu(lanes):
    r = subprocess.run([sys.executable, "bench.py", *COMMON, "--lanes", str(lanes)], cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert REQUIRED <= set(d) and d["n_gpus"] == 1 and d["value"] > 0
    assert d["config"]["global_batch"] == 2 * lanes and d["config"]["parallelism"] == "pp1"
    assert d["config"]["lanes"] == lanes


def test_bench_metrics_out_and_tracing_cpu(tmp_path):
    """--metrics-out appends the result record; EDGELLM_TRACE / EDGELLM_SYNC_DEBUG paths run."""
    path = tmp_path / "m.jsonl"
    env = dict(os.environ, EDGELLM_TRACE="1", EDGELLM_SYNC_DEBUG="1")
    r = subprocess.run([sys.executable, "bench.py", *COMMON, "--lanes", "1", "--metrics-out", str(path)], cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    rec = json.loads(path.read_text().splitlines()[-1])
    assert rec["event"] == "bench" and rec["value"] == d["value"] and rec["metric"] == d["metric"]


@pytest.mark.parametrize("n,lanes,vs", [(2, 1, "on"), (2, 2, "on"), (2, 2, "off"), (3, 2, "on"), (4, 2, "on"),
                                         (8, 1, "on"), (8, 2, "on"), (8, 1, "off")])
def test_bench_pipeline_torchrun_cpu(n, lanes, vs):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(n), *COMMON,
           "--lanes", str(lanes), "--pp-vocab-split", vs]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    # vocab split (default): the head over every rank, one more micro-batch group in flight
    groups = n + 1 if vs == "on" else n
    assert d["vocab_split"] == (vs == "on")
    assert d["n_gpus"] == n and d["config"]["global_batch"] == 2 * groups * lanes and d["value"] > 0
    assert len(d["stage_cost_model_us"]) == n and d["stage_cost_spread"] >= 1.0
    assert d["config"]["parallelism"] == f"pp{n}" and len(d["config"]["partition"]) == n + 1
    # per-rank window statistics from every stage (compute / P2P wait / bubble / bytes per tick)
    assert d["world_size"] == n and len(d["per_rank"]) == n
    for r, st in enumerate(d["per_rank"]):
        assert st["rank"] == r and st["compute_ms_per_tick"] > 0 and 0 <= st["bubble_frac"] <= 1
        assert st["p2p_bytes_per_tick"] > 0
        # host time per tick: posting + completing the exchanges + issuing the compute
        parts = sum(st[f"host_{k}_us_per_tick"] for k in ("post", "finish", "compute"))
        assert st["host_issue_us_per_tick"] > 0 and abs(parts - st["host_issue_us_per_tick"]) < 1e-3 * parts + 1e-6
    assert d["ttft_ms"] > 0 and d["host_issue_us_per_tick_max"] > 0


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_self_launch_cpu(n):
    """``python bench.py --gpus N`` with no torchrun: the script starts its own N rank processes
    and relays rank 0's single JSON line (the command form the driver uses for N = 1)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--device", "cpu", "--model", "tiny:llama", "--steps", "2",
           "--warmup", "1", "--micro-batch", "2", "--prompt-len", "6", "--lanes", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert REQUIRED <= set(d) and d["n_gpus"] == n and d["world_size"] == n and len(d["per_rank"]) == n
    assert d["config"]["parallelism"] == f"pp{n}" and d["value"] > 0


def test_bench_self_launch_killed_rank_cpu(tmp_path):
    """A rank that dies makes the launcher exit non-zero within its grace period instead of
    hanging on the surviving ranks (they block in a collective on the dead peer)."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    # rank 1 kills itself when its pipeline stage starts (fault injection in the stage loop)
    env.update(EDGELLM_FAULT_KILL_RANK="1", EDGELLM_LAUNCH_GRACE_S="5", EDGELLM_WATCHDOG_S="600")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--model", "tiny:llama", "--steps", "2",
           "--warmup", "1", "--micro-batch", "2", "--prompt-len", "6", "--lanes", "1"]
    t0 = time.monotonic()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert time.monotonic() - t0 < 240
    assert "failed" in r.stderr and not [l for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [1, 2])
def test_bench_headinfer_cpu(n):
    """BASELINE config 4 plumbing: --headinfer-heads offloads KV heads in the single-GPU engine and
    in every pipeline stage."""
    args = ["bench.py", "--gpus", str(n), *COMMON, "--headinfer-heads", "1"]
    cmd = [sys.executable, *args] if n == 1 else [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                                                   f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
                                                   "--master-port", str(_port()), *args]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["config"]["headinfer_heads"] == 1 and d["value"] > 0

"""The on-disk INT8 checkpoint end to end (quant/checkpoint.py; the reference quantises at every
load and stores nothing: Code/Quantised Models/models_quant_updated.py:30-38).

* ``edgellm.cli.quantize`` writes the checkpoint of a model quantised exactly as
  ``load_model(..., quant=...)`` does in memory; the directory then works as a model id.
* A stage (whole or half layers) is read without materialising any bf16 projection.
* Under torchrun, pipeline stages loaded from the checkpoint (each rank reads only its layers)
  give the same tokens as the in-memory quantised single-process run.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from test_cli_cpu import _tiny_yaml
from test_pp_cli_cpu import ROOT, _free_port, _rows


def _logits(m, ids):
    from edgellm.models.decoder import AttnCtx
    from edgellm.engine.kv_cache import KVCache
    T = ids.shape[1]
    kv = KVCache(m.cfg, 1, T + 1, m.kv_first, m.last, m.dtype, m.device)
    sp = torch.zeros(1, dtype=torch.int32)
    return m(ids, AttnCtx("prefill", 1, T, sp, sp + T, T, kv.rows(0, 1), m.rope_table()), logits="all").float()


@pytest.mark.parametrize("mode", ["w8a8_smoothquant", "llm_int8"])
def test_quantize_cli_equals_in_memory(tmp_path, mode):
    from edgellm.cli import quantize
    from edgellm.models.registry import load_model
    out = quantize.main(["--model", "tiny:llama", "--quant", mode, "--out", str(tmp_path / "ck"),
                         "--precision", "bf16", "--device", "cpu"])
    meta = json.load(open(os.path.join(out, "quant_config.json")))
    assert meta["mode"] == mode and meta["units"] == [0, 2 * meta["model_config"]["num_layers"]]
    ref, _, _ = load_model("tiny:llama", "bf16", mode, "cpu")
    got, tok, source = load_model(out, "bf16", "none", "cpu")
    assert source.startswith("int8-checkpoint:") and got.quant_mode == mode
    ids = torch.randint(0, ref.cfg.vocab_size, (1, 9), generator=torch.Generator().manual_seed(1))
    assert torch.equal(_logits(got, ids), _logits(ref, ids))


def test_half_layer_stage_from_checkpoint(tmp_path):
    """A sub-layer stage reads exactly its halves; nothing is left on the meta device."""
    from edgellm.models import build_model, tiny
    from edgellm.quant import load_quantized, quantize_model, save_quantized
    cfg = tiny("llama", num_layers=4)
    m = quantize_model(build_model(cfg, dtype=torch.bfloat16, seed=2), "w8a8_smoothquant")
    save_quantized(m, str(tmp_path))
    st = load_quantized(str(tmp_path), units=(3, 8))          # MLP half of layer 1, layers 2-3, head
    assert st.layers[0].attn is None and st.kv_first == 2 and st.has_head and not st.has_embed
    assert all(not t.is_meta for t in st.parameters())
    assert torch.equal(st.layers[0].mlp.down.w_packed, m.layers[1].mlp.down.w_packed)
    assert torch.equal(st.final_norm.weight, m.final_norm.weight)


def test_combine_torchrun_stages_from_checkpoint(tmp_path):
    """2 ranks, each loading only its stage of the checkpoint, answer exactly like the in-memory
    W8A8 single-process run (vote merge, greedy-free sampled decode with the same seeds)."""
    from edgellm.cli import combine, quantize
    ck = quantize.main(["--model", "tiny:llama", "--quant", "w8a8_smoothquant", "--out", str(tmp_path / "ck"),
                        "--precision", "fp32", "--device", "cpu"])
    mem = _tiny_yaml(tmp_path, """
merge: vote
agents:
  - {name: qa, model: "tiny:llama", precision: fp32, quant: w8a8_smoothquant}
""")
    single = tmp_path / "single.jsonl"
    combine.main(["--config", mem, "--devices", "cpu", "--num_samples", "2", "--max_seq", "512",
                  "--metrics_jsonl", str(single)])
    (tmp_path / "ck_yaml").mkdir()
    fromck = _tiny_yaml(tmp_path / "ck_yaml", f"""
merge: vote
agents:
  - {{name: qa, model: "{ck}", precision: fp32}}
""")
    piped = tmp_path / "piped.jsonl"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "-m", "edgellm.cli.combine", "--config", fromck,
           "--devices", "cpu", "--num_samples", "2", "--max_seq", "512", "--metrics_jsonl", str(piped)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "int8-checkpoint:" in r.stdout and "pipelined over 2 ranks" in r.stdout
    a, b = _rows(single), _rows(piped)
    assert len(a) == len(b) == 2
    for x, y in zip(a, b):
        assert x["answers"] == y["answers"] and x["final"] == y["final"]


@pytest.mark.parametrize("source", ["per_stage_calibration", "checkpoint"])
def test_combine_torchrun_4_ranks_half_layers_lanes(tmp_path, source):
    """4 ranks, half-layer stage bounds (``--partition units``: every stage one attention or MLP
    half of the 2-layer tiny Llamas), 2 lanes: the CLI pipeline engine runs the bench's schedule.
    SmoothQuant W8A8 either calibrated PER STAGE over the P2P path (no rank builds the full model)
    or read stage-locally from an int8 checkpoint — answers equal the single-process run."""
    from edgellm.cli import combine, quantize
    agents = """
merge: vote
agents:
  - {name: qa1, model: "tiny:llama", precision: fp32, quant: w8a8_smoothquant}
  - {name: qa2, model: "tiny:llama2", precision: fp32, quant: w8a8_smoothquant}
"""
    mem = _tiny_yaml(tmp_path, agents)
    single = tmp_path / "single.jsonl"
    combine.main(["--config", mem, "--devices", "cpu", "--num_samples", "2", "--max_seq", "512",
                  "--metrics_jsonl", str(single)])
    cfg_path = mem
    if source == "checkpoint":
        cks = [quantize.main(["--model", m, "--quant", "w8a8_smoothquant", "--out", str(tmp_path / f"ck{i}"),
                              "--precision", "fp32", "--device", "cpu"]) for i, m in enumerate(["tiny:llama",
                                                                                              "tiny:llama2"])]
        (tmp_path / "ck_yaml").mkdir()
        cfg_path = _tiny_yaml(tmp_path / "ck_yaml", f"""
merge: vote
agents:
  - {{name: qa1, model: "{cks[0]}", precision: fp32}}
  - {{name: qa2, model: "{cks[1]}", precision: fp32}}
""")
    piped = tmp_path / "piped.jsonl"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "-m", "edgellm.cli.combine", "--config", cfg_path,
           "--devices", "cpu", "--num_samples", "2", "--max_seq", "512", "--metrics_jsonl", str(piped),
           "--partition", "units", "--pp_lanes", "2", "--calib", "stage"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "pipelined over 4 ranks" in r.stdout
    # every stage is one half layer: units [r, r + 1) on rank r
    for rk in range(4):
        assert f"stage {rk}/4 of " in r.stdout and f"units [{rk}, {rk + 1})" in r.stdout
    if source == "checkpoint":
        assert "int8-checkpoint:" in r.stdout
    else:
        assert "(per-stage calibration)" in r.stdout
    a, b = _rows(single), _rows(piped)
    assert len(a) == len(b) == 2
    for x, y in zip(a, b):
        assert x["answers"] == y["answers"] and x["final"] == y["final"]

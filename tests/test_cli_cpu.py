"""Reference-compatibility of the config/CLI layer and end-to-end runs of the entry points on
CPU with tiny random-init agents."""
import logging

import pytest
import yaml

from edgellm.config import add_reference_args, apply_overrides, config_from_dict, load_config

# the two reference YAML layouts (Code/others/config.yaml, Code/C-DAC Server/config_2.yaml)
OTHERS_YAML = """
max_new_tokens: 200
temperature: 0.7
top_k: 50
top_p: 0.9
repetition_penalty: 1.1
dataset_name: sentence-transformers/natural-questions
dataset_split: train[:1000]
dataset_path: /home/research/Desktop/Models
phi_model: /home/research/Desktop/Models/microsoft/phi-2
pythia_model: /home/research/Desktop/Models/EleutherAI/pythia-1b
refiner_model: /home/research/Desktop/Models/meta-llama/Llama-3.2-1B-Instruct
embedder_model: /home/research/Desktop/Models/sentence-transformers/all-MiniLM-L6-v2
"""
CDAC_YAML = """
dataset_name: "sentence-transformers/natural-questions"
dataset_split: "train[:1000]"
dataset_path: "sentence-transformers/natural-questions"
phi_model: "microsoft/phi-2"
pythia_model: "EleutherAI/pythia-1b"
refiner_model: "meta-llama/Llama-3.2-1B-Instruct"
embedder_model: "sentence-transformers/all-MiniLM-L6-v2"
max_new_tokens: 100
temperature: 0.7
top_k: 50
top_p: 0.9
repetition_penalty: 1.2
"""


@pytest.mark.parametrize("text,mnt,rep", [(OTHERS_YAML, 200, 1.1), (CDAC_YAML, 100, 1.2)])
def test_reference_yaml_parses(tmp_path, text, mnt, rep):
    p = tmp_path / "c.yaml"
    p.write_text(text)
    cfg = load_config(str(p))
    assert cfg["max_new_tokens"] == mnt and cfg["repetition_penalty"] == rep
    assert cfg.phi_model.endswith("phi-2") and cfg.dataset_split == "train[:1000]"


def test_cli_override_semantics():
    import argparse
    ap = add_reference_args(argparse.ArgumentParser(), "combiner")
    cfg = config_from_dict(yaml.safe_load(OTHERS_YAML))
    args = ap.parse_args(["--temperature", "0", "--top_k", "30"])
    apply_overrides(cfg, args)                    # non-None wins (combiner rule)
    assert cfg["temperature"] == 0.0 and cfg["top_k"] == 30
    cfg2 = config_from_dict(yaml.safe_load(OTHERS_YAML))
    apply_overrides(cfg2, ap.parse_args(["--temperature", "0"]), legacy_or_overrides=True)
    assert cfg2["temperature"] == 0.7              # the single-model scripts' `or` quirk
    ap1 = add_reference_args(argparse.ArgumentParser(), "single")
    a1 = ap1.parse_args(["--models", "a", "b", "--max_new_tokens", "5"])
    assert a1.models == ["a", "b"]


def _tiny_yaml(tmp_path, extra=""):
    p = tmp_path / "tiny.yaml"
    p.write_text(f"""
max_new_tokens: 4
temperature: 0.7
top_k: 50
top_p: 0.9
repetition_penalty: 1.1
dataset_name: sentence-transformers/natural-questions
dataset_split: train[:3]
phi_model: "tiny:phi"
pythia_model: "tiny:gpt_neox"
refiner_model: "tiny:llama"
embedder_model: "none"
models: ["tiny:llama"]
{extra}
""")
    return str(p)


def test_combine_cli_end_to_end(tmp_path, caplog):
    from edgellm.cli import combine
    prog = tmp_path / "progress.jsonl"
    means = combine.main(["--config", _tiny_yaml(tmp_path), "--devices", "cpu", "--num_samples", "2",
                          "--max_seq", "1024", "--progress", str(prog)])
    assert set(means) >= {"rouge1", "rouge2", "rougeL", "bleu", "bertscore", "cosine", "confidence", "tps"}
    assert means["tps"] > 0
    assert len(prog.read_text().strip().splitlines()) == 2
    # resume: nothing left to do, same means
    again = combine.main(["--config", _tiny_yaml(tmp_path), "--devices", "cpu", "--num_samples", "2",
                          "--max_seq", "1024", "--progress", str(prog)])
    quality = ("rouge1", "rouge2", "rougeL", "bleu", "bertscore", "cosine", "confidence", "tps")
    assert {k: again[k] for k in quality} == {k: means[k] for k in quality}
    # Table-3 efficiency columns measured by the harness (time per sample, memory, agg tok/s)
    assert means["time_per_sample_s"] > 0 and means["agg_tokens_per_s"] > 0 and means["samples"] == 2


def test_combine_batched_split_agents(tmp_path, caplog):
    """Questions decoded 2 per batch, each QA agent's layers split over a 2-stage group
    (parallel.pp_size; the reference's device_map="auto"), int8 KV cache, vote merge."""
    from edgellm.cli import combine
    means = combine.main(["--config", _tiny_yaml(tmp_path), "--devices", "cpu", "--num_samples", "3",
                          "--max_seq", "512", "--batch_size", "2", "--pp_size", "2", "--merge", "vote",
                          "--kv_dtype", "int8"])
    assert means["samples"] == 3 and means["tps"] > 0
    from edgellm.engine import SamplingParams
    from edgellm.parallel.split import SplitLM
    ag = combine.make_agent("a", "tiny:llama", "fp32", "none", "cpu", SamplingParams(max_new_tokens=2),
                            {"pp_size": 2, "batch_size": 2, "max_seq": 64})
    assert isinstance(ag.generator.model, SplitLM) and ag.generator.kv.max_batch == 2


def test_evaluate_headinfer_cli(tmp_path):
    """--headinfer_heads wires HeadInfer offload into the evaluator (one KV head resident)."""
    from edgellm.cli import evaluate
    out = evaluate.main(["--config", _tiny_yaml(tmp_path), "--devices", "cpu", "--num_samples", "1",
                         "--max_seq", "256", "--headinfer_heads", "1", "--prefill_chunk", "16"])
    assert all(v["tps"] > 0 for v in out.values())


def test_combine_vote_and_quant(tmp_path):
    from edgellm.cli import combine
    means = combine.main(["--config", _tiny_yaml(tmp_path), "--devices", "cpu", "--num_samples", "1",
                          "--max_seq", "1024", "--merge", "vote", "--quant", "w8a8_smoothquant", "--no_legacy_decode"])
    assert means["tps"] > 0


def test_evaluate_and_cpu_int8_cli(tmp_path):
    from edgellm.cli import cpu_int8, evaluate
    out = evaluate.main(["--config", _tiny_yaml(tmp_path), "--devices", "cpu", "--num_samples", "1",
                         "--max_seq", "1024"])
    assert "tiny:llama" in out
    means = cpu_int8.main(["--num_samples", "1", "--max_seq", "1024", "--phi_model", "tiny:phi",
                           "--pythia_model", "tiny:gpt_neox", "--refiner_model", "tiny:llama"])
    assert means["tps"] > 0


def test_missing_config_exits(tmp_path):
    from edgellm.cli import combine
    with pytest.raises(SystemExit) as e:
        combine.main(["--config", str(tmp_path / "nope.yaml")])
    assert e.value.code == 1


def test_shipped_configs_parse():
    """Every YAML under configs/ loads through the reference-compatible config loader."""
    import glob
    import os
    from edgellm.config import load_config
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs")
    paths = sorted(glob.glob(os.path.join(root, "*.yaml")))
    assert len(paths) >= 4
    for p in paths:
        cfg = load_config(p)
        assert cfg["top_k"] == 50 and cfg.sampling.max_new_tokens > 0, p
    ns = load_config(os.path.join(root, "north_star.yaml"))
    assert ns.merge == "vote" and len(ns.agents) == 3 and ns.agents[0].gpus == [0, 1]

"""Typed run configuration that accepts the reference's YAML files and CLI flags.

Reference behaviour:
  * flat YAML keys ``max_new_tokens, temperature, top_k, top_p, repetition_penalty,
    dataset_name, dataset_split, dataset_path, phi_model, pythia_model, refiner_model,
    embedder_model`` (Code/others/config.yaml:3-16, Code/C-DAC Server/config_2.yaml:1-14),
    plus ``models:`` for the single-model scripts (Llama_bf16_updated.py:154);
  * CLI flags of the same names (combine_model_fp_updated.py:140-152,
    Llama_bf16_updated.py:138-146);
  * override rule: the combiners use "every non-None CLI value wins"
    (combine_model_fp_updated.py:166-168); the single-model scripts use ``args.x or cfg[x]``
    which silently drops falsy values such as ``--temperature 0``.  We implement the
    non-None rule everywhere (the documented fix) — ``legacy_or_overrides=True`` restores
    the single-model quirk for parity experiments.

New sections (not in the reference): ``parallel``, ``quant``, ``offload``, ``agents``,
``merge``, ``serve``.
"""
from __future__ import annotations

import argparse
import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

REFERENCE_SAMPLING_KEYS = ("max_new_tokens", "temperature", "top_k", "top_p", "repetition_penalty")
REFERENCE_DATA_KEYS = ("dataset_name", "dataset_split", "dataset_path")
REFERENCE_MODEL_KEYS = ("phi_model", "pythia_model", "refiner_model", "embedder_model")


@dataclass
class SamplingConfig:
    # Defaults = Code/others/config.yaml:3-7
    max_new_tokens: int = 200
    temperature: float = 0.7
    top_k: int = 50
    top_p: float = 0.9
    repetition_penalty: float = 1.1
    do_sample: bool = True
    seed: Optional[int] = None


# Fixed refiner sampling parameters (combine_model_fp_updated.py:128-132).
REFINER_SAMPLING = dict(temperature=0.5, top_k=30, top_p=0.9, repetition_penalty=1.1)


@dataclass
class ParallelConfig:
    pp_size: int = 1            # pipeline stages (one process per GPU)
    microbatches: int = 1       # sequences groups in flight through the pipeline
    partition: str = "balanced"  # balanced (by bytes) | units (half-layer decode cost model) | uniform | "8,8,8,8"
    lanes: int = 1              # micro-batches each stage decodes concurrently on HIP streams
    slack: int = 0              # extra ticks per stage hop (1: every P2P hop overlapped with a tick)
    calib: str = "stage"        # SmoothQuant under torchrun: per-stage over P2P | full (every rank)
    vocab_split: bool = True    # torchrun pipelines: LM head split by vocabulary over the stages


@dataclass
class QuantConfig:
    mode: str = "none"          # none | w8a8_smoothquant | llm_int8 | cpu_dynamic
    alpha: float = 0.5          # SmoothQuant migration strength
    outlier_threshold: float = 6.0  # LLM.int8 outlier threshold (bnb default)
    calib_samples: int = 8
    calib_seq_len: int = 128


@dataclass
class OffloadConfig:
    headinfer: bool = False
    gpu_kv_budget_heads: Optional[int] = None   # H_on per layer (None = all on GPU)
    chunk_size: int = 4096                       # chunked-prefill size


@dataclass
class ServeConfig:
    host: str = "0.0.0.0"
    grpc_port: int = 50051      # server.py:16
    rest_port: int = 8000       # rest_api.py:15


@dataclass
class AgentSpec:
    name: str
    model: str
    precision: str = "fp16"
    quant: str = "none"
    gpus: Optional[List[int]] = None


@dataclass
class RunConfig:
    sampling: SamplingConfig = field(default_factory=SamplingConfig)
    dataset_name: str = "sentence-transformers/natural-questions"
    dataset_split: str = "train[:1000]"
    dataset_path: Optional[str] = None
    phi_model: Optional[str] = None
    pythia_model: Optional[str] = None
    refiner_model: Optional[str] = None
    embedder_model: Optional[str] = None
    models: List[str] = field(default_factory=list)
    parallel: ParallelConfig = field(default_factory=ParallelConfig)
    quant: QuantConfig = field(default_factory=QuantConfig)
    offload: OffloadConfig = field(default_factory=OffloadConfig)
    serve: ServeConfig = field(default_factory=ServeConfig)
    agents: List[AgentSpec] = field(default_factory=list)
    merge: str = "refine"       # refine (reference) | vote (north star)
    extra: Dict[str, Any] = field(default_factory=dict)

    # flat reference-style view -------------------------------------------------
    def __getitem__(self, key: str):
        if key in REFERENCE_SAMPLING_KEYS:
            return getattr(self.sampling, key)
        if hasattr(self, key):
            return getattr(self, key)
        return self.extra[key]

    def __setitem__(self, key: str, value):
        if key in REFERENCE_SAMPLING_KEYS or key in ("do_sample", "seed"):
            setattr(self.sampling, key, value)
        elif key in {f.name for f in dataclasses.fields(self)}:
            setattr(self, key, value)
        else:
            self.extra[key] = value

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


def _build_section(cls, data: Optional[dict]):
    if data is None:
        return cls()
    names = {f.name for f in dataclasses.fields(cls)}
    unknown = set(data) - names
    if unknown:
        raise ValueError(f"unknown keys for {cls.__name__}: {sorted(unknown)}")
    return cls(**data)


def config_from_dict(d: dict) -> RunConfig:
    d = dict(d or {})
    cfg = RunConfig()
    sampling = {k: d.pop(k) for k in list(d) if k in REFERENCE_SAMPLING_KEYS or k in ("do_sample", "seed")}
    if "sampling" in d:
        sampling.update(d.pop("sampling") or {})
    cfg.sampling = _build_section(SamplingConfig, sampling)
    for key, cls in (("parallel", ParallelConfig), ("quant", QuantConfig),
                     ("offload", OffloadConfig), ("serve", ServeConfig)):
        if key in d:
            setattr(cfg, key, _build_section(cls, d.pop(key)))
    if "agents" in d:
        cfg.agents = [AgentSpec(**a) for a in (d.pop("agents") or [])]
    for f in dataclasses.fields(RunConfig):
        if f.name in d:
            setattr(cfg, f.name, d.pop(f.name))
    cfg.extra.update(d)
    if isinstance(cfg.models, str):
        cfg.models = [cfg.models]
    return cfg


def load_config(path: Optional[str]) -> RunConfig:
    """Load a YAML config with ``yaml.safe_load`` (as the reference does,
    combine_model_fp_updated.py:162-163).  Accepts both reference files unchanged."""
    if path is None:
        return RunConfig()
    with open(path, "r") as f:
        return config_from_dict(yaml.safe_load(f) or {})


def add_reference_args(parser: argparse.ArgumentParser, style: str = "combiner") -> argparse.ArgumentParser:
    """Register the reference's CLI flags.

    style="combiner": combine_model_fp_updated.py:140-152 (13 flags)
    style="single":   Llama_bf16_updated.py:138-146 (adds --models nargs+)
    """
    parser.add_argument("--config", type=str, default=None, help="Path to YAML config")
    parser.add_argument("--max_new_tokens", type=int)
    parser.add_argument("--temperature", type=float)
    parser.add_argument("--top_k", type=int)
    parser.add_argument("--top_p", type=float)
    parser.add_argument("--repetition_penalty", type=float)
    parser.add_argument("--dataset_name", type=str)
    parser.add_argument("--dataset_split", type=str)
    if style == "single":
        parser.add_argument("--models", nargs="+", help="List of models to evaluate (override YAML)")
    else:
        parser.add_argument("--dataset_path", type=str)
        parser.add_argument("--phi_model", type=str)
        parser.add_argument("--pythia_model", type=str)
        parser.add_argument("--refiner_model", type=str)
        parser.add_argument("--embedder_model", type=str)
    return parser


def apply_overrides(cfg: RunConfig, args: argparse.Namespace, legacy_or_overrides: bool = False) -> RunConfig:
    """Apply CLI overrides. Non-None wins (combine_model_fp_updated.py:166-168).
    With ``legacy_or_overrides`` the single-model ``args.x or cfg[x]`` rule is used
    (Llama_bf16_updated.py:154-161), i.e. falsy CLI values are ignored."""
    for key, value in vars(args).items():
        if key == "config" or value is None:
            continue
        if legacy_or_overrides and not value:
            continue
        cfg[key] = value
    return cfg

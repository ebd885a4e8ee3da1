"""Model architecture descriptions for every family the reference touches.

Families (dims are public HF configs):
  * Llama 2 / 3 / 3.2   — RMSNorm, SwiGLU, full RoPE (llama3 frequency scaling for 3.x), GQA,
                           tied embeddings for 3.2-1B (refiner, combine_model_fp_updated.py:176)
  * GPT-NeoX (Pythia)    — two LayerNorms, parallel residual, partial RoPE (rotary_pct 0.25)
                           (QA agent, combine_model_fp_updated.py:175)
  * Phi-2                — one shared LayerNorm, parallel attn+MLP, partial RoPE (32 of 80),
                           gelu_new, lm_head bias (QA agent, combine_model_fp_updated.py:174)
  * GPT-2                — learned positions, gelu_new (CPU gRPC plumbing config, BASELINE.json)
  * BERT (MiniLM-L6)     — bidirectional encoder used as the sentence embedder
                           (combine_model_fp_updated.py:70-73,179)
A single ``ModelConfig`` describes all decoder families; ``DecoderLM`` interprets the flags.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class ModelConfig:
    arch: str                    # llama | gpt_neox | phi | gpt2 | bert
    vocab_size: int
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    intermediate_size: int
    head_dim: Optional[int] = None
    max_position_embeddings: int = 4096
    norm: str = "rms"            # rms | layer
    norm_eps: float = 1e-5
    act: str = "silu_glu"        # silu_glu | gelu_tanh | gelu
    parallel_residual: bool = False
    shared_input_norm: bool = False   # phi: attn and mlp read the same LayerNorm output
    pos_emb: str = "rope"        # rope | learned | none
    rotary_dim: Optional[int] = None  # partial rotary; None = head_dim
    rope_theta: float = 10000.0
    rope_scaling: Optional[dict] = None  # {"rope_type": "llama3", factor, low_freq_factor, high_freq_factor, original_max_position_embeddings}
    qkv_bias: bool = False
    o_bias: bool = False
    mlp_bias: bool = False
    lm_head_bias: bool = False
    tie_word_embeddings: bool = False
    bos_token_id: Optional[int] = None
    eos_token_id: Optional[int] = None
    name: str = ""

    def __post_init__(self):
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_heads
        if self.rotary_dim is None:
            self.rotary_dim = self.head_dim
        assert self.num_heads % self.num_kv_heads == 0

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def is_glu(self) -> bool:
        return self.act == "silu_glu"

    def num_params(self) -> int:
        h, f = self.hidden_size, self.intermediate_size
        per_layer = h * self.qkv_size + self.q_size * h + (3 if self.is_glu else 2) * h * f
        emb = self.vocab_size * h * (1 if self.tie_word_embeddings else 2)
        return self.num_layers * per_layer + emb

    def layer_bytes(self, weight_bytes: float = 2.0) -> float:
        h, f = self.hidden_size, self.intermediate_size
        return weight_bytes * (h * self.qkv_size + self.q_size * h + (3 if self.is_glu else 2) * h * f)

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


# --------------------------------------------------------------------------- presets
LLAMA3_ROPE_32 = {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                  "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}
LLAMA3_ROPE_8 = dict(LLAMA3_ROPE_32, factor=8.0)

PRESETS = {
    "llama-2-7b": ModelConfig(arch="llama", vocab_size=32000, hidden_size=4096, num_layers=32,
                              num_heads=32, num_kv_heads=32, intermediate_size=11008,
                              max_position_embeddings=4096, norm_eps=1e-5, rope_theta=10000.0,
                              bos_token_id=1, eos_token_id=2, name="llama-2-7b"),
    "llama-3-8b": ModelConfig(arch="llama", vocab_size=128256, hidden_size=4096, num_layers=32,
                              num_heads=32, num_kv_heads=8, intermediate_size=14336,
                              max_position_embeddings=8192, rope_theta=500000.0,
                              bos_token_id=128000, eos_token_id=128001, name="llama-3-8b"),
    "llama-3.2-1b": ModelConfig(arch="llama", vocab_size=128256, hidden_size=2048, num_layers=16,
                                num_heads=32, num_kv_heads=8, intermediate_size=8192,
                                max_position_embeddings=131072, rope_theta=500000.0,
                                rope_scaling=LLAMA3_ROPE_32, tie_word_embeddings=True,
                                bos_token_id=128000, eos_token_id=128009, name="llama-3.2-1b"),
    "phi-2": ModelConfig(arch="phi", vocab_size=51200, hidden_size=2560, num_layers=32,
                         num_heads=32, num_kv_heads=32, intermediate_size=10240,
                         max_position_embeddings=2048, norm="layer", norm_eps=1e-5,
                         act="gelu_tanh", parallel_residual=True, shared_input_norm=True,
                         rotary_dim=32, qkv_bias=True, o_bias=True, mlp_bias=True,
                         lm_head_bias=True, bos_token_id=50256, eos_token_id=50256, name="phi-2"),
    "pythia-1b": ModelConfig(arch="gpt_neox", vocab_size=50304, hidden_size=2048, num_layers=16,
                             num_heads=8, num_kv_heads=8, intermediate_size=8192,
                             max_position_embeddings=2048, norm="layer", norm_eps=1e-5, act="gelu",
                             parallel_residual=True, rotary_dim=64, qkv_bias=True, o_bias=True,
                             mlp_bias=True, bos_token_id=0, eos_token_id=0, name="pythia-1b"),
    "gpt2": ModelConfig(arch="gpt2", vocab_size=50257, hidden_size=768, num_layers=12, num_heads=12,
                        num_kv_heads=12, intermediate_size=3072, max_position_embeddings=1024,
                        norm="layer", norm_eps=1e-5, act="gelu_tanh", pos_emb="learned",
                        qkv_bias=True, o_bias=True, mlp_bias=True, tie_word_embeddings=True,
                        bos_token_id=50256, eos_token_id=50256, name="gpt2"),
    "minilm-l6": ModelConfig(arch="bert", vocab_size=30522, hidden_size=384, num_layers=6,
                             num_heads=12, num_kv_heads=12, intermediate_size=1536,
                             max_position_embeddings=512, norm="layer", norm_eps=1e-12, act="gelu",
                             pos_emb="learned", qkv_bias=True, o_bias=True, mlp_bias=True,
                             name="minilm-l6"),
}
PRESETS["llama2-7b"] = PRESETS["llama-2-7b"]
PRESETS["llama3-8b"] = PRESETS["llama-3-8b"]


def tiny(arch: str = "llama", **kw) -> ModelConfig:
    """Small random-init configs for unit tests (same code paths as the full models)."""
    base = {
        "llama": PRESETS["llama-3.2-1b"].replace(vocab_size=512, hidden_size=128, num_layers=2,
                                                 num_heads=4, num_kv_heads=2, intermediate_size=256,
                                                 max_position_embeddings=512, name="tiny-llama"),
        "llama2": PRESETS["llama-2-7b"].replace(vocab_size=512, hidden_size=128, num_layers=2,
                                                num_heads=4, num_kv_heads=4, intermediate_size=256,
                                                max_position_embeddings=512, name="tiny-llama2"),
        "phi": PRESETS["phi-2"].replace(vocab_size=512, hidden_size=160, num_layers=2, num_heads=2,
                                        num_kv_heads=2, intermediate_size=320, rotary_dim=32,
                                        max_position_embeddings=512, name="tiny-phi"),
        "gpt_neox": PRESETS["pythia-1b"].replace(vocab_size=512, hidden_size=128, num_layers=2,
                                                 num_heads=2, num_kv_heads=2, head_dim=64,
                                                 intermediate_size=256, rotary_dim=16,
                                                 max_position_embeddings=512, name="tiny-neox"),
        "gpt2": PRESETS["gpt2"].replace(vocab_size=512, hidden_size=128, num_layers=2, num_heads=2,
                                        num_kv_heads=2, intermediate_size=256,
                                        max_position_embeddings=512, name="tiny-gpt2"),
        "bert": PRESETS["minilm-l6"].replace(vocab_size=512, hidden_size=64, num_layers=2,
                                             num_heads=2, num_kv_heads=2, intermediate_size=128,
                                             max_position_embeddings=128, name="tiny-bert"),
    }[arch]
    return base.replace(**kw) if kw else base


def get_config(name: str) -> ModelConfig:
    key = name.lower()
    if key in PRESETS:
        return PRESETS[key]
    if os.path.isdir(name):
        return from_hf_dir(name)
    raise KeyError(f"unknown model '{name}'; presets: {sorted(PRESETS)}")


def to_hf_config(cfg: ModelConfig) -> dict:
    """ModelConfig -> a Hugging Face ``config.json`` dict (inverse of ``from_hf_config``)."""
    common = dict(vocab_size=cfg.vocab_size, max_position_embeddings=cfg.max_position_embeddings,
                  tie_word_embeddings=cfg.tie_word_embeddings, bos_token_id=cfg.bos_token_id,
                  eos_token_id=cfg.eos_token_id, torch_dtype="bfloat16")
    partial = cfg.rotary_dim / cfg.head_dim
    if cfg.arch == "llama":
        return dict(common, model_type="llama", architectures=["LlamaForCausalLM"], hidden_size=cfg.hidden_size,
                    intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_layers,
                    num_attention_heads=cfg.num_heads, num_key_value_heads=cfg.num_kv_heads,
                    head_dim=cfg.head_dim, rms_norm_eps=cfg.norm_eps, rope_theta=cfg.rope_theta,
                    rope_scaling=cfg.rope_scaling, attention_bias=cfg.qkv_bias, mlp_bias=cfg.mlp_bias,
                    hidden_act="silu")
    if cfg.arch == "gpt_neox":
        return dict(common, model_type="gpt_neox", architectures=["GPTNeoXForCausalLM"],
                    hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                    num_hidden_layers=cfg.num_layers, num_attention_heads=cfg.num_heads,
                    layer_norm_eps=cfg.norm_eps, rotary_pct=partial, rotary_emb_base=cfg.rope_theta,
                    use_parallel_residual=cfg.parallel_residual,
                    hidden_act="gelu" if cfg.act == "gelu" else "gelu_new", attention_bias=cfg.qkv_bias)
    if cfg.arch == "phi":
        return dict(common, model_type="phi", architectures=["PhiForCausalLM"], hidden_size=cfg.hidden_size,
                    intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_layers,
                    num_attention_heads=cfg.num_heads, num_key_value_heads=cfg.num_kv_heads,
                    layer_norm_eps=cfg.norm_eps, partial_rotary_factor=partial, rope_theta=cfg.rope_theta,
                    hidden_act="gelu_new")
    if cfg.arch == "gpt2":
        return dict(common, model_type="gpt2", architectures=["GPT2LMHeadModel"], n_embd=cfg.hidden_size,
                    n_layer=cfg.num_layers, n_head=cfg.num_heads, n_inner=cfg.intermediate_size,
                    n_positions=cfg.max_position_embeddings, layer_norm_epsilon=cfg.norm_eps,
                    activation_function="gelu_new")
    raise ValueError(f"no HF config mapping for {cfg.arch}")


def from_hf_dir(path: str) -> ModelConfig:
    with open(os.path.join(path, "config.json")) as f:
        return from_hf_config(json.load(f))


def _rope_params(c: dict, default_theta: float, default_partial: float = 1.0):
    """(theta, partial_rotary_factor, scaling) from either the transformers-5 ``rope_parameters``
    dict or the older flat keys (rope_theta / rotary_emb_base / rotary_pct / rope_scaling)."""
    rp = dict(c.get("rope_parameters") or {})
    theta = rp.get("rope_theta", c.get("rope_theta", c.get("rotary_emb_base", default_theta)))
    partial = rp.get("partial_rotary_factor",
                     c.get("partial_rotary_factor", c.get("rotary_pct", default_partial)))
    scaling = c.get("rope_scaling")
    if rp.get("rope_type", "default") not in ("default", None):
        scaling = {k: v for k, v in rp.items() if k not in ("rope_theta", "partial_rotary_factor")}
    if scaling and scaling.get("rope_type", scaling.get("type")) in ("default", None):
        scaling = None
    return float(theta), float(partial), scaling


def from_hf_config(c: dict) -> ModelConfig:
    """Map a Hugging Face ``config.json`` onto ModelConfig."""
    mt = c.get("model_type")
    eos = c.get("eos_token_id")
    if isinstance(eos, list):
        eos = eos[0]
    if mt in ("llama", "mistral"):
        h, nh = c["hidden_size"], c["num_attention_heads"]
        theta, _, scaling = _rope_params(c, 10000.0)
        return ModelConfig(arch="llama", vocab_size=c["vocab_size"], hidden_size=h,
                           num_layers=c["num_hidden_layers"], num_heads=nh,
                           num_kv_heads=c.get("num_key_value_heads", nh),
                           intermediate_size=c["intermediate_size"],
                           head_dim=c.get("head_dim") or h // nh,
                           max_position_embeddings=c.get("max_position_embeddings", 4096),
                           norm_eps=c.get("rms_norm_eps", 1e-5), rope_theta=theta,
                           rope_scaling=scaling,
                           qkv_bias=c.get("attention_bias", False), o_bias=c.get("attention_bias", False),
                           mlp_bias=c.get("mlp_bias", False),
                           tie_word_embeddings=c.get("tie_word_embeddings", False),
                           bos_token_id=c.get("bos_token_id"), eos_token_id=eos,
                           name=c.get("_name_or_path", "llama"))
    if mt == "gpt_neox":
        h, nh = c["hidden_size"], c["num_attention_heads"]
        hd = h // nh
        theta, partial, scaling = _rope_params(c, 10000.0, 0.25)
        return ModelConfig(arch="gpt_neox", vocab_size=c["vocab_size"], hidden_size=h,
                           num_layers=c["num_hidden_layers"], num_heads=nh, num_kv_heads=nh,
                           intermediate_size=c["intermediate_size"],
                           max_position_embeddings=c.get("max_position_embeddings", 2048),
                           norm="layer", norm_eps=c.get("layer_norm_eps", 1e-5),
                           act="gelu" if c.get("hidden_act", "gelu") == "gelu" else "gelu_tanh",
                           parallel_residual=c.get("use_parallel_residual", True),
                           rotary_dim=int(hd * partial), rope_theta=theta, rope_scaling=scaling,
                           qkv_bias=c.get("attention_bias", True), o_bias=c.get("attention_bias", True),
                           mlp_bias=True, tie_word_embeddings=c.get("tie_word_embeddings", False),
                           bos_token_id=c.get("bos_token_id"), eos_token_id=eos, name="gpt_neox")
    if mt == "phi":
        h, nh = c["hidden_size"], c["num_attention_heads"]
        hd = h // nh
        theta, partial, scaling = _rope_params(c, 10000.0, 0.4)
        return ModelConfig(arch="phi", vocab_size=c["vocab_size"], hidden_size=h,
                           num_layers=c["num_hidden_layers"], num_heads=nh,
                           num_kv_heads=c.get("num_key_value_heads") or nh,
                           intermediate_size=c["intermediate_size"],
                           max_position_embeddings=c.get("max_position_embeddings", 2048),
                           norm="layer", norm_eps=c.get("layer_norm_eps", 1e-5), act="gelu_tanh",
                           parallel_residual=True, shared_input_norm=True,
                           rotary_dim=int(hd * partial), rope_theta=theta, rope_scaling=scaling,
                           qkv_bias=True, o_bias=True,
                           mlp_bias=True, lm_head_bias=True,
                           tie_word_embeddings=c.get("tie_word_embeddings", False),
                           bos_token_id=c.get("bos_token_id"), eos_token_id=eos, name="phi")
    if mt == "gpt2":
        h, nh = c["n_embd"], c["n_head"]
        return ModelConfig(arch="gpt2", vocab_size=c["vocab_size"], hidden_size=h,
                           num_layers=c["n_layer"], num_heads=nh, num_kv_heads=nh,
                           intermediate_size=c.get("n_inner") or 4 * h,
                           max_position_embeddings=c.get("n_positions", 1024), norm="layer",
                           norm_eps=c.get("layer_norm_epsilon", 1e-5), act="gelu_tanh",
                           pos_emb="learned", qkv_bias=True, o_bias=True, mlp_bias=True,
                           tie_word_embeddings=True, bos_token_id=c.get("bos_token_id"),
                           eos_token_id=eos, name="gpt2")
    if mt == "bert":
        h, nh = c["hidden_size"], c["num_attention_heads"]
        return ModelConfig(arch="bert", vocab_size=c["vocab_size"], hidden_size=h,
                           num_layers=c["num_hidden_layers"], num_heads=nh, num_kv_heads=nh,
                           intermediate_size=c["intermediate_size"],
                           max_position_embeddings=c.get("max_position_embeddings", 512),
                           norm="layer", norm_eps=c.get("layer_norm_eps", 1e-12), act="gelu",
                           pos_emb="learned", qkv_bias=True, o_bias=True, mlp_bias=True, name="bert")
    raise ValueError(f"unsupported model_type {mt!r}")

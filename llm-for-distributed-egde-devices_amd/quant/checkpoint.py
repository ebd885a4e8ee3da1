"""On-disk quantised checkpoint format (new capability: the reference quantises only at load
time and never stores INT8 weights — SURVEY §5.4).

A directory with
  quant_config.json   {"format": "edgellm-int8", "version": 1, "mode": ..., "alpha": ...,
                       "threshold": ..., "smoothing": "folded", "model_config": {...}}
  model.safetensors   per quantised projection ``<p>``:
                        <p>.qweight  int8 [N, K]  canonical row-major (not the MFMA packing —
                                                  packing is a load-time layout choice)
                        <p>.w_scale  f32 [N]      per-output-channel scale   (w8a8 modes)
                        <p>.SCB      f32 [N]      per-row absmax, bnb naming  (llm_int8)
                        <p>.bias     bf16 [N]
                      every other parameter in bf16 under its global edgellm name
                      (norm weights already carry the folded SmoothQuant factors)
                      ``smooth.<p>`` f32 [K] the factors themselves (informational)
Stage-aware: ``load_quantized(..., first, last)`` reads only that stage's tensors.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch

from ..models.configs import ModelConfig
from ..models.decoder import DecoderLM, global_named_parameters
from .linear import LLMInt8Linear, W8A8Linear, enable_fused_glu

FORMAT = "edgellm-int8"
VERSION = 1
_PROJ = (("attn", "qkv"), ("attn", "o"), ("mlp", "up"), ("mlp", "down"))


def is_quantized_checkpoint(path: Optional[str]) -> bool:
    """A directory written by ``save_quantized`` (``quant_config.json`` of this format)."""
    if not path or not os.path.isdir(path):
        return False
    f = os.path.join(path, "quant_config.json")
    if not os.path.exists(f):
        return False
    with open(f) as fh:
        return json.load(fh).get("format") == FORMAT


def checkpoint_quant_mode(path: str) -> str:
    """The quantisation mode a checkpoint was written in (``quant_config.json`` "mode")."""
    with open(os.path.join(path, "quant_config.json")) as f:
        return json.load(f).get("mode", "none") or "none"


def checkpoint_config(path: str) -> ModelConfig:
    with open(os.path.join(path, "quant_config.json")) as f:
        return ModelConfig(**json.load(f)["model_config"])


@torch.no_grad()
def save_quantized(model: DecoderLM, path: str, extra: Optional[dict] = None) -> None:
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    mode = getattr(model, "quant_mode", "none")
    tensors = {}
    quant_names = set()
    for layer in model.layers:
        for a, b in _PROJ:
            parent = getattr(layer, a)
            if parent is None:                   # half layer of a sub-layer stage
                continue
            mod = getattr(parent, b)
            p = f"layers.{layer.idx}.{a}.{b}"
            bias = mod.bias
            if isinstance(mod, W8A8Linear):          # canonical [gate | up] row order on disk
                q, sc, bias = mod.canonical()
                tensors[p + ".qweight"] = q.cpu()
                tensors[p + ".w_scale"] = sc.cpu()
            elif isinstance(mod, LLMInt8Linear):
                tensors[p + ".qweight"] = mod.weight_i8.cpu()
                tensors[p + ".SCB"] = mod.SCB.cpu()
            else:
                continue
            quant_names.add(p)
            if bias is not None:
                tensors[p + ".bias"] = bias.cpu()
    for name, prm in global_named_parameters(model):
        if any(name.startswith(q + ".") for q in quant_names):
            continue
        tensors[name] = prm.detach().cpu().contiguous()
    for name, s in (getattr(model, "smooth_factors", None) or {}).items():   # keys: global layer index
        tensors["smooth." + name] = s.float().contiguous()
    save_file(tensors, os.path.join(path, "model.safetensors"))
    meta = {"format": FORMAT, "version": VERSION, "mode": mode, "model_config": model.cfg.to_dict(),
            "smoothing": "folded" if mode == "w8a8_smoothquant" else "none", "first": model.first,
            "last": model.last, "units": list(getattr(model, "units", (2 * model.first, 2 * model.last)))}
    meta.update(extra or {})
    with open(os.path.join(path, "quant_config.json"), "w") as f:
        json.dump(meta, f, indent=2)


@torch.no_grad()
def load_quantized(path: str, device=None, first: int = 0, last: Optional[int] = None,
                   dtype=torch.bfloat16, units: Optional[tuple] = None) -> DecoderLM:
    """The stage [first, last) (or half-layer ``units``) of a quantised checkpoint.  Only that
    stage's tensors are read, and no bf16 copy of a projection is ever materialised: the model is
    built on the meta device and every tensor is created from the file on ``device`` (a pipeline
    rank of a 7B model reads its ~1/P of 7 GB int8 instead of building and calibrating 13.5 GB)."""
    from safetensors import safe_open
    with open(os.path.join(path, "quant_config.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path} is not an {FORMAT} checkpoint")
    cfg = ModelConfig(**meta["model_config"])
    mode = meta["mode"]
    saved = tuple(meta.get("units") or (2 * meta.get("first", 0), 2 * meta.get("last", cfg.num_layers)))
    if units is not None:
        model = DecoderLM.from_units(cfg, units[0], units[1], dtype=dtype, device="meta").eval()
    else:
        model = DecoderLM(cfg, dtype=dtype, device="meta", first=first, last=last).eval()
    ua, ub = model.units
    assert saved[0] <= ua and ub <= saved[1], f"checkpoint holds units {saved}, stage needs {model.units}"
    device = torch.device(device) if device is not None else torch.device("cpu")
    with safe_open(os.path.join(path, "model.safetensors"), framework="pt") as sf:
        keys = set(sf.keys())
        for layer in model.layers:
            for a, b in _PROJ:
                parent = getattr(layer, a)
                if parent is None:
                    continue
                p = f"layers.{layer.idx}.{a}.{b}"
                if p + ".qweight" not in keys:
                    continue
                lin = getattr(parent, b)
                bias = sf.get_tensor(p + ".bias").to(device) if p + ".bias" in keys else None
                q = sf.get_tensor(p + ".qweight").to(device)
                if p + ".SCB" in keys:
                    new = LLMInt8Linear(lin.in_features, lin.out_features, bias is not None,
                                        meta.get("threshold", 6.0), device=device, dtype=dtype)
                    new.load_int8(q, sf.get_tensor(p + ".SCB").to(device), bias)
                else:
                    new = W8A8Linear(lin.in_features, lin.out_features, bias is not None, device=device, dtype=dtype)
                    new.load_int8(q, sf.get_tensor(p + ".w_scale").to(device), bias)
                setattr(parent, b, new)
        # every remaining (meta) parameter straight from the file onto the device
        for name, prm in list(global_named_parameters(model)):
            src = name
            if src not in keys and name == "lm_head.weight" and cfg.tie_word_embeddings:
                src = "embed"
            t = sf.get_tensor(src).to(device=device, dtype=prm.dtype)
            _set_param(model, _local_name(model, name), t)
    left = [n for n, t in list(model.named_parameters()) + list(model.named_buffers()) if t.is_meta]
    assert not left, f"checkpoint left {left[:4]} unloaded"
    model.quant_mode = mode
    if mode in ("w8a8_smoothquant", "w8a8"):
        enable_fused_glu(model)
    return model


def load_head_rows(path: str, v0: int, v1: int, device=None, dtype=torch.bfloat16):
    """Rows [v0, v1) of a quantised checkpoint's (16-bit) LM head and its bias, read as a slice
    (a vocab shard of the head, parallel/vocab_head.py: no rank reads the whole matrix)."""
    from safetensors import safe_open
    cfg = checkpoint_config(path)
    with safe_open(os.path.join(path, "model.safetensors"), framework="pt") as sf:
        keys = set(sf.keys())
        assert "lm_head.qweight" not in keys, "vocab split: 16-bit LM head only"
        name = "lm_head.weight" if "lm_head.weight" in keys or not cfg.tie_word_embeddings else "embed"
        w = sf.get_slice(name)[v0:v1].to(device=device, dtype=dtype)
        b = sf.get_slice("lm_head.bias")[v0:v1].to(device=device, dtype=dtype) if "lm_head.bias" in keys else None
    return w, b


def _local_name(model: DecoderLM, global_name: str) -> str:
    if global_name.startswith("layers."):
        _, idx, rest = global_name.split(".", 2)
        return f"layers.{int(idx) - model.first}.{rest}"
    return global_name


def _set_param(model: torch.nn.Module, name: str, t: torch.Tensor) -> None:
    mod = model
    parts = name.split(".")
    for p in parts[:-1]:
        mod = getattr(mod, p)
    mod._parameters[parts[-1]] = torch.nn.Parameter(t, requires_grad=False)

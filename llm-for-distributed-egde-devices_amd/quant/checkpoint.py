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


@torch.no_grad()
def save_quantized(model: DecoderLM, path: str, extra: Optional[dict] = None) -> None:
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    mode = getattr(model, "quant_mode", "none")
    tensors = {}
    quant_names = set()
    for layer in model.layers:
        for a, b in _PROJ:
            mod = getattr(getattr(layer, a), b)
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
            "last": model.last}
    meta.update(extra or {})
    with open(os.path.join(path, "quant_config.json"), "w") as f:
        json.dump(meta, f, indent=2)


@torch.no_grad()
def load_quantized(path: str, device=None, first: int = 0, last: Optional[int] = None,
                   dtype=torch.bfloat16) -> DecoderLM:
    from safetensors import safe_open
    with open(os.path.join(path, "quant_config.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path} is not an {FORMAT} checkpoint")
    cfg = ModelConfig(**meta["model_config"])
    mode = meta["mode"]
    model = DecoderLM(cfg, dtype=dtype, device=device, first=first, last=last).eval()
    with safe_open(os.path.join(path, "model.safetensors"), framework="pt") as sf:
        keys = set(sf.keys())
        for layer in model.layers:
            for a, b in _PROJ:
                p = f"layers.{layer.idx}.{a}.{b}"
                if p + ".qweight" not in keys:
                    continue
                lin = getattr(getattr(layer, a), b)
                bias = sf.get_tensor(p + ".bias").to(device) if p + ".bias" in keys else None
                q = sf.get_tensor(p + ".qweight").to(device)
                if p + ".SCB" in keys:
                    new = LLMInt8Linear(lin.in_features, lin.out_features, bias is not None,
                                        meta.get("threshold", 6.0), device=device, dtype=dtype)
                    new.load_int8(q, sf.get_tensor(p + ".SCB").to(device), bias)
                else:
                    new = W8A8Linear(lin.in_features, lin.out_features, bias is not None, device=device, dtype=dtype)
                    new.load_int8(q, sf.get_tensor(p + ".w_scale").to(device), bias)
                setattr(getattr(layer, a), b, new)
        for name, prm in global_named_parameters(model):
            src = name
            if src not in keys and name == "lm_head.weight" and cfg.tie_word_embeddings:
                src = "embed"
            prm.copy_(sf.get_tensor(src).to(device=prm.device, dtype=prm.dtype))
    model.quant_mode = mode
    if mode in ("w8a8_smoothquant", "w8a8"):
        enable_fused_glu(model)
    return model

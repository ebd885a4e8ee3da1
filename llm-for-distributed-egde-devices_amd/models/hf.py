"""Hugging Face checkpoint interop.

Reads ``save_pretrained`` directories — including the reference downloader's
``BASE_DIR/<org>_<name>`` layout (Code/C-DAC Server/download.py:20-24) — by streaming
safetensors shards tensor by tensor onto the target device (no full-model host copy), and
converts HF parameter names/layouts into edgellm's fused layout:

  Llama   q/k/v_proj -> attn.qkv (rows [q|k|v]); gate/up_proj -> mlp.up (rows [gate|up])
  NeoX    query_key_value is interleaved per head ([h][q,k,v][D]) -> de-interleaved [q|k|v]
  Phi-2   q/k/v_proj (+bias) -> attn.qkv; dense -> attn.o; fc1/fc2; final_layernorm; lm_head(+bias)
  GPT-2   Conv1D weights are [in, out] -> transposed; c_attn is already [q|k|v]

Only layers [first, last) are materialised, so a pipeline stage loads its own slice.
Safetensors only (never pickle).  ``*.bin`` checkpoints are read with
``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import glob
import json
import os
import re
from typing import Dict, Iterator, Optional, Tuple

import torch

from .configs import ModelConfig, from_hf_config
from .decoder import DecoderLM


def _iter_checkpoint(path: str) -> Iterator[Tuple[str, torch.Tensor]]:
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if files:
        from safetensors import safe_open
        for f in files:
            with safe_open(f, framework="pt") as sf:
                for k in sf.keys():
                    yield k, sf.get_tensor(k)
        return
    for f in sorted(glob.glob(os.path.join(path, "*.bin"))):
        sd = torch.load(f, map_location="cpu", weights_only=True)
        yield from sd.items()


_LAYER_RE = re.compile(r"(?:model\.layers|gpt_neox\.layers|transformer\.h)\.(\d+)\.(.*)")


def convert_hf_tensors(cfg: ModelConfig, items: Iterator[Tuple[str, torch.Tensor]], first: int = 0,
                       last: Optional[int] = None) -> Dict[str, torch.Tensor]:
    """HF (name, tensor) stream -> edgellm global parameter names (``layers.<global i>...``)."""
    last = cfg.num_layers if last is None else last
    out: Dict[str, torch.Tensor] = {}
    pend: Dict[int, Dict[str, torch.Tensor]] = {}
    hq, hk, d = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
    arch = cfg.arch
    for name, t in items:
        m = _LAYER_RE.match(name)
        if m:
            i = int(m.group(1))
            if not (first <= i < last):
                continue
            pend.setdefault(i, {})[m.group(2)] = t
            continue
        if arch in ("llama", "phi"):
            if name == "model.embed_tokens.weight":
                out["embed"] = t
            elif name in ("model.norm.weight", "model.final_layernorm.weight"):
                out["final_norm.weight"] = t
            elif name == "model.final_layernorm.bias":
                out["final_norm.bias"] = t
            elif name == "lm_head.weight":
                out["lm_head.weight"] = t
            elif name == "lm_head.bias":
                out["lm_head.bias"] = t
        elif arch == "gpt_neox":
            mp = {"gpt_neox.embed_in.weight": "embed", "gpt_neox.final_layer_norm.weight": "final_norm.weight",
                  "gpt_neox.final_layer_norm.bias": "final_norm.bias", "embed_out.weight": "lm_head.weight",
                  "lm_head.weight": "lm_head.weight"}
            if name in mp:
                out[mp[name]] = t
        elif arch == "gpt2":
            mp = {"transformer.wte.weight": "embed", "wte.weight": "embed", "transformer.wpe.weight": "pos_embed",
                  "wpe.weight": "pos_embed", "transformer.ln_f.weight": "final_norm.weight",
                  "transformer.ln_f.bias": "final_norm.bias", "ln_f.weight": "final_norm.weight",
                  "ln_f.bias": "final_norm.bias"}
            if name in mp:
                out[mp[name]] = t
    for i, p in pend.items():
        pre = f"layers.{i}."
        if arch == "llama":
            out[pre + "norm1.weight"] = p["input_layernorm.weight"]
            out[pre + "norm2.weight"] = p["post_attention_layernorm.weight"]
            out[pre + "attn.qkv.weight"] = torch.cat([p["self_attn.q_proj.weight"], p["self_attn.k_proj.weight"],
                                                      p["self_attn.v_proj.weight"]], 0)
            if "self_attn.q_proj.bias" in p:
                out[pre + "attn.qkv.bias"] = torch.cat([p["self_attn.q_proj.bias"], p["self_attn.k_proj.bias"],
                                                        p["self_attn.v_proj.bias"]], 0)
            out[pre + "attn.o.weight"] = p["self_attn.o_proj.weight"]
            out[pre + "mlp.up.weight"] = torch.cat([p["mlp.gate_proj.weight"], p["mlp.up_proj.weight"]], 0)
            out[pre + "mlp.down.weight"] = p["mlp.down_proj.weight"]
        elif arch == "phi":
            out[pre + "norm1.weight"] = p["input_layernorm.weight"]
            out[pre + "norm1.bias"] = p["input_layernorm.bias"]
            for w in ("weight", "bias"):
                out[pre + f"attn.qkv.{w}"] = torch.cat([p[f"self_attn.q_proj.{w}"], p[f"self_attn.k_proj.{w}"],
                                                        p[f"self_attn.v_proj.{w}"]], 0)
                out[pre + f"attn.o.{w}"] = p[f"self_attn.dense.{w}"]
                out[pre + f"mlp.up.{w}"] = p[f"mlp.fc1.{w}"]
                out[pre + f"mlp.down.{w}"] = p[f"mlp.fc2.{w}"]
        elif arch == "gpt_neox":
            for w in ("weight", "bias"):
                out[pre + f"norm1.{w}"] = p[f"input_layernorm.{w}"]
                out[pre + f"norm2.{w}"] = p[f"post_attention_layernorm.{w}"]
                qkv = p[f"attention.query_key_value.{w}"]
                qkv = qkv.view(hq, 3, d, *qkv.shape[1:]).transpose(0, 1).reshape(qkv.shape)
                out[pre + f"attn.qkv.{w}"] = qkv
                out[pre + f"attn.o.{w}"] = p[f"attention.dense.{w}"]
                out[pre + f"mlp.up.{w}"] = p[f"mlp.dense_h_to_4h.{w}"]
                out[pre + f"mlp.down.{w}"] = p[f"mlp.dense_4h_to_h.{w}"]
        elif arch == "gpt2":
            for w in ("weight", "bias"):
                out[pre + f"norm1.{w}"] = p[f"ln_1.{w}"]
                out[pre + f"norm2.{w}"] = p[f"ln_2.{w}"]
            out[pre + "attn.qkv.weight"] = p["attn.c_attn.weight"].t()
            out[pre + "attn.qkv.bias"] = p["attn.c_attn.bias"]
            out[pre + "attn.o.weight"] = p["attn.c_proj.weight"].t()
            out[pre + "attn.o.bias"] = p["attn.c_proj.bias"]
            out[pre + "mlp.up.weight"] = p["mlp.c_fc.weight"].t()
            out[pre + "mlp.up.bias"] = p["mlp.c_fc.bias"]
            out[pre + "mlp.down.weight"] = p["mlp.c_proj.weight"].t()
            out[pre + "mlp.down.bias"] = p["mlp.c_proj.bias"]
        else:
            raise ValueError(f"no HF converter for {arch}")
    return out


@torch.no_grad()
def load_into(model: DecoderLM, tensors: Dict[str, torch.Tensor], strict: bool = True) -> DecoderLM:
    from .decoder import global_named_parameters
    params = dict(global_named_parameters(model))
    missing = []
    for name, p in params.items():
        t = tensors.get(name)
        if t is None and name == "lm_head.weight" and model.cfg.tie_word_embeddings and "embed" in tensors:
            t = tensors["embed"]          # tied head on a stage without the embedding
        if t is None:
            missing.append(name)
            continue
        assert tuple(t.shape) == tuple(p.shape), f"{name}: {tuple(t.shape)} vs {tuple(p.shape)}"
        p.copy_(t.to(p.dtype))
    if strict and missing:
        raise KeyError(f"checkpoint is missing {missing[:8]}{'...' if len(missing) > 8 else ''}")
    return model


def load_hf_model(path: str, dtype=torch.bfloat16, device=None, first: int = 0,
                  last: Optional[int] = None) -> DecoderLM:
    with open(os.path.join(path, "config.json")) as f:
        cfg = from_hf_config(json.load(f))
    model = DecoderLM(cfg, dtype=dtype, device=device, first=first, last=last).eval()
    tensors = convert_hf_tensors(cfg, _iter_checkpoint(path), first, model.last)
    return load_into(model, tensors)


def from_hf_module(hf_model, cfg: Optional[ModelConfig] = None, dtype=torch.bfloat16, device=None) -> DecoderLM:
    """Build an edgellm model from an in-memory HF model (tests / conversion)."""
    cfg = cfg or from_hf_config(hf_model.config.to_dict())
    model = DecoderLM(cfg, dtype=dtype, device=device).eval()
    return load_into(model, convert_hf_tensors(cfg, iter(hf_model.state_dict().items())))


def export_hf_tensors(model: DecoderLM) -> Dict[str, torch.Tensor]:
    """edgellm parameters -> HF names/layouts (inverse of ``convert_hf_tensors``; full model only)."""
    from .decoder import global_named_parameters
    cfg = model.cfg
    assert model.first == 0 and model.last == cfg.num_layers, "export needs the whole model"
    p = {k: v.detach() for k, v in global_named_parameters(model)}
    hq, hk, d = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
    qs, ks = hq * d, hk * d
    out: Dict[str, torch.Tensor] = {}
    arch = cfg.arch
    top = {"llama": ("model.embed_tokens.weight", "model.norm", "lm_head"),
           "phi": ("model.embed_tokens.weight", "model.final_layernorm", "lm_head"),
           "gpt_neox": ("gpt_neox.embed_in.weight", "gpt_neox.final_layer_norm", "embed_out"),
           "gpt2": ("transformer.wte.weight", "transformer.ln_f", None)}[arch]
    out[top[0]] = p["embed"]
    for w in ("weight", "bias"):
        if f"final_norm.{w}" in p:
            out[f"{top[1]}.{w}"] = p[f"final_norm.{w}"]
    if top[2] and not cfg.tie_word_embeddings:
        for w in ("weight", "bias"):
            if f"lm_head.{w}" in p:
                out[f"{top[2]}.{w}"] = p[f"lm_head.{w}"]
    if arch == "gpt2":
        out["transformer.wpe.weight"] = p["pos_embed"]
    for i in range(cfg.num_layers):
        s = f"layers.{i}."
        g = lambda n: p.get(s + n)  # noqa: E731
        if arch in ("llama", "phi"):
            h = f"model.layers.{i}."
            for w in ("weight", "bias"):
                qkv = g(f"attn.qkv.{w}")
                if qkv is not None:
                    out[h + f"self_attn.q_proj.{w}"], out[h + f"self_attn.k_proj.{w}"], \
                        out[h + f"self_attn.v_proj.{w}"] = qkv[:qs], qkv[qs:qs + ks], qkv[qs + ks:]
                if g(f"norm1.{w}") is not None:
                    out[h + f"input_layernorm.{w}"] = g(f"norm1.{w}")
            if arch == "llama":
                out[h + "post_attention_layernorm.weight"] = g("norm2.weight")
                out[h + "self_attn.o_proj.weight"] = g("attn.o.weight")
                up = g("mlp.up.weight")
                out[h + "mlp.gate_proj.weight"], out[h + "mlp.up_proj.weight"] = up[:cfg.intermediate_size], \
                    up[cfg.intermediate_size:]
                out[h + "mlp.down_proj.weight"] = g("mlp.down.weight")
            else:
                for w in ("weight", "bias"):
                    out[h + f"self_attn.dense.{w}"] = g(f"attn.o.{w}")
                    out[h + f"mlp.fc1.{w}"] = g(f"mlp.up.{w}")
                    out[h + f"mlp.fc2.{w}"] = g(f"mlp.down.{w}")
        elif arch == "gpt_neox":
            h = f"gpt_neox.layers.{i}."
            for w in ("weight", "bias"):
                out[h + f"input_layernorm.{w}"] = g(f"norm1.{w}")
                out[h + f"post_attention_layernorm.{w}"] = g(f"norm2.{w}")
                qkv = g(f"attn.qkv.{w}")
                out[h + f"attention.query_key_value.{w}"] = \
                    qkv.reshape(3, hq, d, *qkv.shape[1:]).transpose(0, 1).reshape(qkv.shape).contiguous()
                out[h + f"attention.dense.{w}"] = g(f"attn.o.{w}")
                out[h + f"mlp.dense_h_to_4h.{w}"] = g(f"mlp.up.{w}")
                out[h + f"mlp.dense_4h_to_h.{w}"] = g(f"mlp.down.{w}")
        elif arch == "gpt2":
            h = f"transformer.h.{i}."
            for w in ("weight", "bias"):
                out[h + f"ln_1.{w}"] = g(f"norm1.{w}")
                out[h + f"ln_2.{w}"] = g(f"norm2.{w}")
            for ours, theirs in (("attn.qkv", "attn.c_attn"), ("attn.o", "attn.c_proj"), ("mlp.up", "mlp.c_fc"),
                                 ("mlp.down", "mlp.c_proj")):
                out[h + f"{theirs}.weight"] = g(f"{ours}.weight").t()
                out[h + f"{theirs}.bias"] = g(f"{ours}.bias")
    return {k: v.contiguous() for k, v in out.items()}


def save_hf_model(model: DecoderLM, path: str, shard_bytes: int = 4 << 30) -> str:
    """Write ``config.json`` + safetensors shards readable by both edgellm and transformers."""
    from safetensors.torch import save_file
    from .configs import to_hf_config
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(to_hf_config(model.cfg), f, indent=2)
    tensors = export_hf_tensors(model)
    shards, cur, size = [], {}, 0
    for k, v in tensors.items():
        if cur and size + v.numel() * v.element_size() > shard_bytes:
            shards.append(cur)
            cur, size = {}, 0
        cur[k] = v.cpu()
        size += v.numel() * v.element_size()
    shards.append(cur)
    index = {}
    for n, sh in enumerate(shards):
        fn = "model.safetensors" if len(shards) == 1 else f"model-{n + 1:05d}-of-{len(shards):05d}.safetensors"
        save_file(sh, os.path.join(path, fn), metadata={"format": "pt"})
        index.update({k: fn for k in sh})
    if len(shards) > 1:
        with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {}, "weight_map": index}, f)
    return path


def resolve_model_dir(name_or_path: str, base_dir: Optional[str] = None) -> Optional[str]:
    """Find a checkpoint directory the way the reference's scripts/downloader lay them out:
    a direct path, ``base_dir/<name>`` (Llama_bf16_updated.py:165-167) or
    ``base_dir/<org>_<name>`` (download.py:22)."""
    cands = [name_or_path]
    if base_dir:
        cands += [os.path.join(base_dir, name_or_path), os.path.join(base_dir, name_or_path.replace("/", "_"))]
    for c in cands:
        if os.path.isfile(os.path.join(c, "config.json")):
            return c
    return None

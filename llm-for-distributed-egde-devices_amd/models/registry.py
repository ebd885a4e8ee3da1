"""Resolve the reference's model names/paths to a loaded edgellm model + tokenizer.

The reference loads ``AutoModelForCausalLM.from_pretrained(path, torch_dtype=..., device_map="auto")``
from local ``save_pretrained`` dirs or HF ids (Code/others/config.yaml:13-16, config_2.yaml:5-8).
Here: a checkpoint directory that exists locally is loaded (safetensors, streamed); otherwise —
no network, SURVEY Appendix B — the architecture named by the id is random-initialised (logged
loudly) so every pipeline still runs end to end on synthetic weights.
"""
from __future__ import annotations

import zlib
from typing import Optional, Tuple

import torch

from ..utils.log import get_logger
from ..utils.tokenizer import ByteTokenizer, load_tokenizer
from .configs import ModelConfig, PRESETS, get_config
from .decoder import DecoderLM, build_model
from .hf import load_hf_model, resolve_model_dir

log = get_logger("registry")

_ALIASES = [("phi-2", "phi-2"), ("phi2", "phi-2"), ("pythia-1b", "pythia-1b"), ("pythia", "pythia-1b"),
            ("llama-3.2-1b", "llama-3.2-1b"), ("llama3.2-1b", "llama-3.2-1b"), ("llama-2-7b", "llama-2-7b"),
            ("llama2-7b", "llama-2-7b"), ("llama-3-8b", "llama-3-8b"), ("meta-llama-3-8b", "llama-3-8b"),
            ("llama3-8b", "llama-3-8b"), ("gpt2", "gpt2"), ("minilm", "minilm-l6")]


def preset_for(name: str) -> Optional[str]:
    n = name.lower().replace("_", "-")
    if n.startswith("tiny:"):
        return n
    if n in PRESETS:
        return n
    for key, preset in _ALIASES:
        if key in n:
            return preset
    return None


def precision_dtype(precision: str, device, quant: str = "none") -> torch.dtype:
    """torch dtype of a model's 16-bit tensors for the reference's ``precision`` flag
    (combine_model_fp_updated.py:32-34: fp16 unless "bf16"; phi2-pythia_fp_updated.py:32).  The
    GPU runs fp16 and bf16 models on their own kernel instantiations (fp16 MFMA GEMV / attention,
    fp16 norms and RoPE).  Quantised models (``quant`` != none) keep bf16 activations on the GPU:
    the INT8 GEMM epilogues write bf16."""
    p = (precision or "bf16").lower()
    dev = torch.device(device) if device is not None else torch.device("cpu")
    want = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}.get(p, torch.bfloat16)
    if dev.type == "cuda":
        if quant not in (None, "none") and want != torch.bfloat16:
            log.info(f"precision {p} with --quant {quant}: the INT8 kernels run bf16 activations")
            return torch.bfloat16
        if want == torch.float32:
            log.info("precision fp32 on the GPU: the HIP kernels run 16-bit; using bf16")
            return torch.bfloat16
    return want


def quantized_checkpoint_dir(name_or_path: str, base_dir: Optional[str] = None) -> Optional[str]:
    """The directory of an edgellm int8 checkpoint (``edgellm.cli.quantize``) named by the model
    id, directly or under ``base_dir``; None otherwise."""
    import os
    from ..quant.checkpoint import is_quantized_checkpoint
    for c in (name_or_path, os.path.join(base_dir, name_or_path) if base_dir else None,
              os.path.join(base_dir, name_or_path.replace("/", "_")) if base_dir else None):
        if c and is_quantized_checkpoint(c):
            return c
    return None


def load_model(name_or_path: str, precision: str = "bf16", quant: str = "none", device=None,
               base_dir: Optional[str] = None, first: int = 0, last: Optional[int] = None,
               config_override: Optional[ModelConfig] = None, units: Optional[tuple] = None
               ) -> Tuple[DecoderLM, object, str]:
    """Returns (model, tokenizer, source) with source "checkpoint:<dir>", "int8-checkpoint:<dir>"
    (an edgellm quantised checkpoint: its stage is read directly, already quantised — ``quant``
    is then the checkpoint's own mode) or "random-init:<preset>".  ``units``: a half-layer stage."""
    qdir = quantized_checkpoint_dir(name_or_path, base_dir)
    if qdir is not None:
        from ..quant.checkpoint import checkpoint_quant_mode, load_quantized
        # the checkpoint's own INT8 mode sets the activation dtype (bf16 epilogues on the GPU),
        # whatever --quant says (callers pass quant="none" for a checkpoint)
        dtype = precision_dtype(precision, device, checkpoint_quant_mode(qdir))
        model = load_quantized(qdir, device=device, first=first, last=last, dtype=dtype, units=units)
        if quant not in (None, "none", model.quant_mode):
            log.warning(f"{qdir} holds {model.quant_mode} weights: --quant {quant} ignored")
        return model, load_tokenizer(qdir, model.cfg.vocab_size), f"int8-checkpoint:{qdir}"
    dtype = precision_dtype(precision, device, quant)
    path = resolve_model_dir(name_or_path, base_dir)
    if path is not None:
        assert units is None, "half-layer stages of HF checkpoints: load the whole layers"
        model = load_hf_model(path, dtype=dtype, device=device, first=first, last=last)
        tok = load_tokenizer(path, model.cfg.vocab_size)
        source = f"checkpoint:{path}"
    else:
        preset = preset_for(name_or_path)
        if preset is None and config_override is None:
            raise FileNotFoundError(f"no checkpoint at '{name_or_path}' and no architecture preset matches it")
        if config_override is not None:
            cfg = config_override
        elif preset.startswith("tiny:"):     # "tiny:<arch>" test/smoke architectures
            from .configs import tiny
            cfg = tiny(preset.split(":", 1)[1].replace("gpt-neox", "gpt_neox"))
        else:
            cfg = get_config(preset)
        seed = zlib.crc32(name_or_path.encode()) & 0xFFFF
        model = build_model(cfg, dtype=dtype, device=device, first=first, last=last, seed=seed, units=units)
        tok = ByteTokenizer(max(259, cfg.vocab_size))
        source = f"random-init:{cfg.name or preset}"
        log.warning(f"No checkpoint for '{name_or_path}': using random-init {cfg.name or preset} weights "
                    f"(synthetic; quality metrics are meaningless)")
    if quant and quant != "none":
        from ..quant import quantize_model
        calib = None
        if quant == "w8a8_smoothquant" and model.has_embed:
            text = ("Question: when did the first world war begin and which countries fought in it? Answer: "
                    "The First World War began in 1914 after the assassination of Archduke Franz Ferdinand.")
            ids = tok.encode(text)[:64]
            calib = torch.tensor([[i % model.cfg.vocab_size for i in ids]], device=model.device)
        model = quantize_model(model, "w8a8" if (quant == "w8a8_smoothquant" and calib is None) else quant, calib)
    return model, tok, source

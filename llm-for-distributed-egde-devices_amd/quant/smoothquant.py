"""SmoothQuant calibration / smoothing and whole-model quantisation.

SmoothQuant (Xiao et al., 2211.10438 — listed in the reference's paper library but never
implemented there) migrates activation outliers into the weights with a
per-input-channel factor  s_j = max|X_j|^alpha / max|W_j|^(1-alpha):  X' = X / s, W' = W * s.
Every division of X is FOLDED into the producer so inference costs nothing extra:

  qkv input   = norm1 output      -> norm1.weight (and LayerNorm bias) /= s
  up input    = norm2 output      -> norm2.weight /= s      (phi: norm1, joint s for qkv+up)
  o input     = attention output  -> v rows of the qkv weight /= s   (attention is linear in V;
                                     with GQA s is shared by the q heads of a kv group)
  down input  = silu(gate) * up   -> up rows of the fused [gate|up] weight /= s  (GLU only;
                                     GELU is not homogeneous, so non-GLU down is not smoothed)

The lm_head and embeddings stay bf16 (as bitsandbytes/HF also skip the output head).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from ..models.decoder import AttnCtx, DecoderLM
from ..models.layers import Linear
from .linear import CPUDynamicLinear, LLMInt8Linear, W8A8Linear, enable_fused_glu

QUANT_MODES = ("none", "w8a8_smoothquant", "w8a8", "llm_int8", "cpu_dynamic")


@torch.no_grad()
def collect_act_absmax(model: DecoderLM, calib_ids: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Per-input-channel max|x| of every projection input over calibration tokens [N, T]."""
    from ..engine.kv_cache import KVCache
    stats: Dict[str, torch.Tensor] = {}
    hooks = []
    for name, mod in model.named_modules():
        if isinstance(mod, Linear) and ".attn." in f".{name}" or (isinstance(mod, Linear) and ".mlp." in f".{name}"):
            def hook(m, inp, name=name):
                x = inp[0]
                a = x.detach().reshape(-1, x.shape[-1]).abs().amax(0).float()
                stats[name] = torch.maximum(stats[name], a) if name in stats else a
            hooks.append(mod.register_forward_pre_hook(hook))
    try:
        N, T = calib_ids.shape
        kv = KVCache(model.cfg, 1, T, first_layer=model.first, last_layer=model.last, dtype=model.dtype,
                     device=calib_ids.device)
        rope = model.rope_table(calib_ids.device)
        for i in range(N):
            sp = torch.zeros(1, dtype=torch.int32, device=calib_ids.device)
            ctx = AttnCtx("prefill", 1, T, sp, sp + T, T, kv, rope)
            model(calib_ids[i:i + 1], ctx)
    finally:
        for h in hooks:
            h.remove()
    return stats


def _smooth_factor(x_absmax: torch.Tensor, w_colmax: torch.Tensor, alpha: float) -> torch.Tensor:
    s = x_absmax.clamp_min(1e-5).pow(alpha) / w_colmax.clamp_min(1e-5).pow(1 - alpha)
    return s.clamp_min(1e-5)


@torch.no_grad()
def smooth_model_(model: DecoderLM, stats: Dict[str, torch.Tensor], alpha: float = 0.5) -> Dict[str, torch.Tensor]:
    """Fold SmoothQuant factors into norms / producer weights in place.  Returns the per-linear
    factors (the quantiser multiplies W's input columns by them)."""
    cfg = model.cfg
    hq, hk, d = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
    g = hq // hk
    factors: Dict[str, torch.Tensor] = {}
    for j, layer in enumerate(model.layers):
        pre = f"layers.{j}."                       # stats are keyed by local module names
        gpre = f"layers.{layer.idx}."               # factors by GLOBAL layer index
        # half layers (a sub-layer stage): every fold below stays inside its own half
        qkv, o = (layer.attn.qkv, layer.attn.o) if layer.attn is not None else (None, None)
        up, down = (layer.mlp.up, layer.mlp.down) if layer.mlp is not None else (None, None)
        if qkv is None:
            stats = {k: v for k, v in stats.items() if not k.startswith(pre + "attn.")}
        if up is None:
            stats = {k: v for k, v in stats.items() if not k.startswith(pre + "mlp.")}
        # ---- qkv (+ up when phi shares the norm)
        xs = stats.get(pre + "attn.qkv")
        if xs is not None:
            dev = qkv.weight.device
            wmax = qkv.weight.float().abs().amax(0)
            if cfg.shared_input_norm:
                xs = torch.maximum(xs, stats.get(pre + "mlp.up", xs))
                wmax = torch.maximum(wmax, up.weight.float().abs().amax(0))
            s = _smooth_factor(xs.to(dev), wmax, alpha)
            _fold_norm(layer.norm1, s)
            factors[gpre + "attn.qkv"] = s
            if cfg.shared_input_norm:
                factors[gpre + "mlp.up"] = s
        # ---- up (separate norm2)
        if not cfg.shared_input_norm and pre + "mlp.up" in stats:
            dev = up.weight.device
            s = _smooth_factor(stats[pre + "mlp.up"].to(dev), up.weight.float().abs().amax(0), alpha)
            _fold_norm(layer.norm2, s)
            factors[gpre + "mlp.up"] = s
        # ---- o: fold into v rows (shared across the q heads of a kv group)
        if pre + "attn.o" in stats:
            dev = qkv.weight.device
            xs = stats[pre + "attn.o"].to(dev).view(hk, g, d).amax(1)              # [hk, d]
            wm = o.weight.float().abs().amax(0).view(hk, g, d).amax(1)
            s_kv = _smooth_factor(xs, wm, alpha)                                    # [hk, d]
            vs = cfg.q_size + cfg.kv_size
            qkv.weight[vs:] = (qkv.weight[vs:].float() / s_kv.reshape(-1, 1)).to(qkv.weight.dtype)
            if qkv.bias is not None:
                qkv.bias[vs:] = (qkv.bias[vs:].float() / s_kv.reshape(-1)).to(qkv.bias.dtype)
            factors[gpre + "attn.o"] = s_kv[:, None, :].expand(hk, g, d).reshape(-1)
        # ---- down: fold into the up half of the GLU weight
        if cfg.is_glu and pre + "mlp.down" in stats:
            dev = up.weight.device
            f = cfg.intermediate_size
            s = _smooth_factor(stats[pre + "mlp.down"].to(dev), down.weight.float().abs().amax(0), alpha)
            up.weight[f:] = (up.weight[f:].float() / s[:, None]).to(up.weight.dtype)
            if up.bias is not None:
                up.bias[f:] = (up.bias[f:].float() / s).to(up.bias.dtype)
            factors[gpre + "mlp.down"] = s
    return factors


def _fold_norm(norm, s: torch.Tensor):
    norm.weight.copy_((norm.weight.float() / s).to(norm.weight.dtype))
    if norm.bias is not None:
        norm.bias.copy_((norm.bias.float() / s).to(norm.bias.dtype))


def synthetic_calibration(cfg, n: int = 4, T: int = 64, device=None, seed: int = 0) -> torch.Tensor:
    """Random token ids for calibrating random-init models (no datasets offline)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, cfg.vocab_size, (n, T), generator=g).to(device)


@torch.no_grad()
def quantize_model(model: DecoderLM, mode: str, calib_ids: Optional[torch.Tensor] = None, alpha: float = 0.5,
                   threshold: float = 6.0, factors: Optional[Dict[str, torch.Tensor]] = None) -> DecoderLM:
    """Replace every attention/MLP projection of ``model`` in place.

    mode: "w8a8_smoothquant" (calibrate + smooth + W8A8), "w8a8" (no smoothing),
          "llm_int8" (bitsandbytes-compatible), "cpu_dynamic" (torch qint8 dynamic, CPU).
    ``factors`` (keyed by GLOBAL layer index) = smoothing already folded into this model's norms
    (pipeline stages cut from a calibrated full model, see ``smoothquant_stage``)."""
    assert mode in QUANT_MODES, mode
    if mode == "none":
        return model
    if factors is None:
        factors = {}
        if mode == "w8a8_smoothquant":
            if calib_ids is None:
                calib_ids = synthetic_calibration(model.cfg, device=model.device)
            stats = collect_act_absmax(model, calib_ids.to(model.device))
            factors = smooth_model_(model, stats, alpha)
    for layer in model.layers:
        gpre = f"layers.{layer.idx}."
        for parent, attr, key in ((layer.attn, "qkv", "attn.qkv"), (layer.attn, "o", "attn.o"),
                                  (layer.mlp, "up", "mlp.up"), (layer.mlp, "down", "mlp.down")):
            if parent is None:                 # half layer of a sub-layer pipeline stage
                continue
            lin = getattr(parent, attr)
            if mode in ("w8a8_smoothquant", "w8a8"):
                s = factors.get(gpre + key)
                new = W8A8Linear.from_float(lin, s.to(lin.weight.device) if s is not None else None)
            elif mode == "llm_int8":
                new = LLMInt8Linear.from_float(lin, threshold)
            else:
                new = CPUDynamicLinear(lin)
            setattr(parent, attr, new)
    model.quant_mode = mode
    if mode in ("w8a8_smoothquant", "w8a8"):
        enable_fused_glu(model)
    if mode == "w8a8_smoothquant":
        model.smooth_factors = {k: v.detach().cpu() for k, v in factors.items()
                                if model.first <= int(k.split(".")[1]) < model.last}
    return model


@torch.no_grad()
def quantize_head(model: DecoderLM) -> DecoderLM:
    """Optional W8A8 LM head (per-output-channel int8 weights, per-token int8 activations fused
    into the final norm): halves the head's 2 V H bytes, the largest single GEMM of a decode step
    (262 MB bf16 at Llama-2-7B), which is what the pipeline's last stage carries on top of its
    layers.  Off by default — the reference, like bitsandbytes and SmoothQuant, keeps the head in
    16 bits.  A tied head (Llama-3.2-1B: the 525 MB embedding doubles as the head) gets an int8 copy
    of the embedding matrix as its head; the embedding lookup keeps the bf16 table."""
    if model.lm_head is not None and not isinstance(model.lm_head, W8A8Linear):
        model.lm_head = W8A8Linear.from_float(model.lm_head, None)
        model.head_quant = "w8a8"
    elif model.lm_head is None and model.has_head and model.has_embed:
        from types import SimpleNamespace
        tied = SimpleNamespace(weight=model.embed, bias=None, in_features=model.cfg.hidden_size,
                               out_features=model.cfg.vocab_size)
        model.lm_head = W8A8Linear.from_float(tied, None)
        model.head_quant = "w8a8"
    return model


@torch.no_grad()
def smoothquant_stage(full: DecoderLM, first: int, last: int, calib_ids: torch.Tensor, alpha: float = 0.5,
                      device=None, units=None) -> DecoderLM:
    """Calibrate + smooth the FULL model once, then cut layers [first, last) (or the half-layer
    units ``units=(ua, ub)``) into a W8A8 stage.  Every pipeline split (1/2/4/8, whole or
    sub-layer boundaries) therefore gets bit-identical quantised weights for a layer."""
    from ..models.decoder import global_named_parameters
    stats = collect_act_absmax(full, calib_ids.to(full.device))
    factors = smooth_model_(full, stats, alpha)
    if units is not None:
        stage = DecoderLM.from_units(full.cfg, units[0], units[1], dtype=full.dtype,
                                     device=device or full.device).eval()
    else:
        stage = DecoderLM(full.cfg, dtype=full.dtype, device=device or full.device, first=first, last=last).eval()
    src = dict(global_named_parameters(full))
    for name, p in global_named_parameters(stage):
        if name == "lm_head.weight" and name not in src:
            name = "embed"                     # tied head on a head-only stage
        p.copy_(src[name])
    return quantize_model(stage, "w8a8_smoothquant", factors=factors)


@torch.no_grad()
def smoothquant_stage_p2p(cfg, calib_ids: torch.Tensor, recv_prev, send_next, first: int = 0,
                          last: Optional[int] = None, units=None, dtype=torch.bfloat16, device=None,
                          seed: Optional[int] = 0, alpha: float = 0.5, build=None) -> DecoderLM:
    """SmoothQuant for ONE pipeline stage without the full model on this rank: the stage's bf16
    layers are built (``build()``, default random-init ``build_model`` seeded by global parameter
    name), the calibration activations come from the previous stage over the pipeline's P2P path
    (``recv_prev(shape, dtype) -> tensor``; stage 0 embeds ``calib_ids`` [N, T]), this stage's
    projection inputs are measured, its bf16 outputs go on to the next stage (``send_next``),
    and then it is smoothed and quantised.  The stage sees exactly the activations it sees at
    inference, so a rank never materialises layers it does not own (peak build memory ~ 1/P of
    the full model's); with fp32 activations the factors equal ``smoothquant_stage``'s bit for bit."""
    from ..engine.kv_cache import KVCache
    from ..models.decoder import build_model
    stage = build() if build is not None else build_model(cfg, dtype=dtype, device=device, first=first, last=last,
                                                         seed=seed, units=units)
    dev = stage.device
    N, T = calib_ids.shape
    H = cfg.hidden_size
    hidden = None if stage.has_embed else recv_prev((N, T, H), stage.dtype)
    stats: Dict[str, torch.Tensor] = {}
    hooks = []
    for name, mod in stage.named_modules():
        if isinstance(mod, Linear) and (".attn." in f".{name}" or ".mlp." in f".{name}"):
            def hook(m, inp, name=name):
                x = inp[0]
                a = x.detach().reshape(-1, x.shape[-1]).abs().amax(0).float()
                stats[name] = torch.maximum(stats[name], a) if name in stats else a
            hooks.append(mod.register_forward_pre_hook(hook))
    outs = []
    try:
        kv = KVCache(cfg, 1, T, first_layer=getattr(stage, "kv_first", stage.first), last_layer=stage.last,
                     dtype=stage.dtype, device=dev)
        rope = stage.rope_table(dev)
        for i in range(N):
            sp = torch.zeros(1, dtype=torch.int32, device=dev)
            ctx = AttnCtx("prefill", 1, T, sp, sp + T, T, kv, rope)
            out = stage(calib_ids[i:i + 1].to(dev) if stage.has_embed else None, ctx,
                        hidden=None if hidden is None else hidden[i].to(dev))
            if not stage.has_head:
                outs.append(out.view(T, H))
    finally:
        for h in hooks:
            h.remove()
    if not stage.has_head:
        send_next(torch.stack(outs).contiguous())
    factors = smooth_model_(stage, stats, alpha)
    return quantize_model(stage, "w8a8_smoothquant", factors=factors)


def is_graph_safe(model: nn.Module) -> bool:
    return all(getattr(m, "graph_safe", True) for m in model.modules())

"""One decoder implementation for Llama 2/3/3.2, GPT-NeoX (Pythia), Phi-2 and GPT-2.

Replaces the reference's ``AutoModelForCausalLM`` + accelerate stack
(Code/Base Models/combine_model_fp_updated.py:32-42).  Per-layer data flow:

  sequential (llama, gpt2):  h = x + res ; a = attn(norm1(h)) ; h2 = a + h ; out = mlp(norm2(h2))
  parallel   (phi):          h = x + res ; n = norm(h)        ; out = attn(n) + mlp(n)
  parallel   (gpt_neox):     h = x + res ; out = attn(norm1(h)) + mlp(norm2(h))

The residual add is fused into the next norm kernel (``ops.rms_norm(x, w, eps, residual)``),
so each layer returns ``(x, residual)`` and never materialises the sum separately.
Weights use fused layouts: qkv = [q heads | k heads | v heads] rows, GLU up = [gate | up] rows.

The KV cache is head-major ``[B, Hkv, S, D]`` per layer (edgellm.engine.kv_cache) so that
HeadInfer-style head offload is a contiguous copy.  A model can be cut into pipeline stages
(``stage(first, last)``): a stage owns layers [first, last), the embedding if first == 0 and
the head if last == num_layers; it exchanges a single bf16 hidden tensor with its neighbours.
"""
from __future__ import annotations

import math
import os
import zlib
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn

from .. import ops
from ..utils import tracing
from .configs import ModelConfig
from .layers import Linear, Norm, PartialSum, PendingLN, PendingNorm, QAct, act_fn, quant_if

# split-K slices of the bf16 o / down decode GEMVs (0 = off); N = 2048-4096 outputs have only
# 128-256 tiles, so two slices put every CU to work
BF16_SPLIT_K = int(os.environ.get("EDGELLM_BF16_SPLITK", "2"))


@dataclass
class AttnCtx:
    """Per-forward attention metadata.

    mode       "prefill" (T tokens per sequence, causal over cache + new) or "decode" (T == 1)
    start_pos  int32 [B]: cache position of the first new token of each sequence
    seq_lens   int32 [B]: valid cache length after this forward (decode attention)
    max_len    host-side upper bound of seq_lens (sizes the split-K grid; graph-capture bucket)
    kv         object with ``layer(i) -> (k [B,Hkv,S,D], v)``, i = global layer index
    """
    mode: str
    B: int
    T: int
    start_pos: torch.Tensor
    seq_lens: torch.Tensor
    max_len: int
    kv: object
    rope: Optional[torch.Tensor] = None
    causal: bool = True
    attn_hook: Optional[object] = None   # HeadInfer offload manager (edgellm.offload)
    # ragged prefill: int64 [B] index (within the T new tokens) of each row's last real token; rows
    # are right-padded to T, so a real token never attends to a pad (causal) and the pads' cache
    # entries lie past the row's length, where decode overwrites them before any read
    last_pos: Optional[torch.Tensor] = None
    # batch-1 decode through the persistent one-launch engine (engine/b1_engine.py) when eligible
    b1: bool = False

    def last_rows(self, device) -> torch.Tensor:
        """Flat row indices [B] of each sequence's last real token in a [B*T, H] activation."""
        last = self.last_pos.to(device) if self.last_pos is not None else self.T - 1
        return torch.arange(self.B, device=device) * self.T + last


class Attention(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int, dtype, device):
        super().__init__()
        self.cfg, self.layer_idx = cfg, layer_idx
        self.qkv = Linear(cfg.hidden_size, cfg.qkv_size, cfg.qkv_bias, dtype, device)
        self.o = Linear(cfg.q_size, cfg.hidden_size, cfg.o_bias, dtype, device)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)

    def forward(self, x, ctx: AttnCtx):
        cfg = self.cfg
        qkv = self.qkv(x)                                   # [B*T, qkv]
        k_cache, v_cache = ctx.kv.layer(self.layer_idx)
        rot = cfg.rotary_dim if cfg.pos_emb == "rope" else 0
        if ctx.attn_hook is not None:
            # int8 offload (HeadInferKV kv_dtype="int8") hands decode output to a W8A8 o-proj as
            # per-(token, 64) int8, like the resident int8 path
            quant = ctx.mode == "decode" and getattr(ctx.attn_hook, "q8", False) and self.o.takes_quantized_input \
                and cfg.head_dim % 64 == 0 and getattr(self.o, "group_scales_ok", lambda m: m <= 64)(ctx.B)
            attn = ctx.attn_hook.attention(self.layer_idx, qkv, ctx, self.scale, rot, quant) if quant else \
                ctx.attn_hook.attention(self.layer_idx, qkv, ctx, self.scale, rot)
            if isinstance(attn, QAct):
                return self.o(attn)
        elif getattr(ctx.kv, "quantized", False):
            return self._forward_kv8(qkv, ctx, k_cache, v_cache, rot)
        elif ctx.mode == "decode":
            # one launch: RoPE + KV append + attention (+ per-group int8 output for a W8A8 o-proj)
            # per-(token, 64) int8 output feeds the decode GEMV (<= 64 rows, <= 128 for the shapes
            # with 128-row kernels); larger batches take bf16 attention output and per-token quant
            quant = self.o.takes_quantized_input and cfg.head_dim % 64 == 0 and \
                getattr(self.o, "group_scales_ok", lambda m: m <= 64)(ctx.B)
            out, s = ops.decode_attention_fused(qkv.view(ctx.B, -1), ctx.start_pos, ctx.rope if rot else None,
                                                k_cache, v_cache, ctx.seq_lens, cfg.num_heads, self.scale,
                                                ctx.max_len, rot, quant)
            if quant:
                return self.o(QAct(out, s))
            attn = out
        else:
            q = ops.rope_kv_write(qkv, ctx.start_pos, ctx.rope if rot else None, k_cache, v_cache,
                                  cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, rot)  # [B,T,Hq,D]
            attn = ops.prefill_attention(q, k_cache, v_cache, ctx.start_pos, self.scale, ctx.causal)
        attn = attn.reshape(ctx.B * ctx.T, cfg.q_size)
        return self.o(quant_if(attn, self.o))


    def _forward_kv8(self, qkv, ctx: AttnCtx, k_cache, v_cache, rot: int):
        """int8 KV cache (engine.kv_cache, kv_dtype="int8").  Decode: one launch for RoPE +
        quantising append + attention over the int8 cache.  Prefill: RoPE writes the rotated bf16
        k / v of the new tokens (plus, when start > 0, the history dequantised by one kernel) into a
        per-stream scratch shared by all layers, the prefill attention reads it, and the new rows are
        quantised into the cache.

        Precision: the prompt's own tokens attend to their unquantised bf16 k / v during prefill;
        every later read (decode steps, the next chunk's history) sees the int8-rounded values."""
        cfg = self.cfg
        ks, vs = ctx.kv.layer_scales(self.layer_idx)
        if ctx.mode == "decode":
            quant = self.o.takes_quantized_input and getattr(self.o, "group_scales_ok", lambda m: m <= 64)(ctx.B)
            out, s = ops.decode_attention_fused_i8(qkv.view(ctx.B, -1), ctx.start_pos, ctx.rope if rot else None,
                                                   k_cache, v_cache, ks, vs, ctx.seq_lens, cfg.num_heads, self.scale,
                                                   ctx.max_len, rot, quant)
            if quant:
                return self.o(QAct(out, s))
            attn = out
        else:
            B, T, S = ctx.B, ctx.T, ctx.max_len
            hist = S - T                                  # host bound of the cached prefix
            if hasattr(ctx.kv, "prefill_scratch"):
                kb, vb = ctx.kv.prefill_scratch(B, S, qkv.dtype, qkv.device)
            else:
                kb = torch.empty(B, cfg.num_kv_heads, S, cfg.head_dim, dtype=qkv.dtype, device=qkv.device)
                vb = torch.empty_like(kb)
            if hist > 0:
                ops.kv_dequant(k_cache, ks, kb, hist)
                ops.kv_dequant(v_cache, vs, vb, hist)
            q = ops.rope_kv_write(qkv, ctx.start_pos, ctx.rope if rot else None, kb, vb, cfg.num_heads,
                                  cfg.num_kv_heads, cfg.head_dim, rot)
            ops.kv_quant_append(kb, ctx.start_pos, T, k_cache, ks)
            ops.kv_quant_append(vb, ctx.start_pos, T, v_cache, vs)
            attn = ops.prefill_attention(q, kb, vb, ctx.start_pos, self.scale, ctx.causal)
        attn = attn.reshape(ctx.B * ctx.T, cfg.q_size)
        return self.o(quant_if(attn, self.o))


# prefill SwiGLU in the gate_up GEMM epilogue (EDGELLM_PREFILL_GLU=0: GEMM + blocked activation kernel)
_PREFILL_GLU = os.environ.get("EDGELLM_PREFILL_GLU", "1") != "0"


class MLP(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        self.act = cfg.act
        up_out = 2 * cfg.intermediate_size if cfg.is_glu else cfg.intermediate_size
        self.up = Linear(cfg.hidden_size, up_out, cfg.mlp_bias, dtype, device)
        self.down = Linear(cfg.intermediate_size, cfg.hidden_size, cfg.mlp_bias, dtype, device)

    def forward(self, x, add=None):
        """``add``: the attention branch of a parallel-residual block, added to the down
        projection's output (in its decode GEMV's epilogue)."""
        if isinstance(x, PendingLN):
            if self.act in ("gelu_tanh", "gelu") and type(self.up) is Linear:
                return self.down(self.up.forward_ln(x, act=self.act), add=add)     # 16-bit up + GELU
            if x.quant and self.act in ("gelu_tanh", "gelu") and hasattr(self.up, "geluq"):
                return self.down(self.up.geluq(x, self.act), add=add)              # W8A8 up + GELU + quant
            if not getattr(self.up, "takes_pending_x", False):
                x = x.materialize()
            else:                                      # LLM.int8: the norm in the up projection's prologue
                if self.act in ("gelu_tanh", "gelu") and hasattr(self.up, "gelu_fused"):
                    h = self.up.gelu_fused(x, self.act)        # + the GELU in its epilogue
                    if h is not None:
                        return self.down(h, add=add)
                if self.act == "silu_glu" and hasattr(self.up, "glu_norm"):
                    h = self.up.glu_norm(x)            # + the SwiGLU in its epilogue
                    if h is not None:
                        return self.down(h, add=add)
                return self.down(act_fn(self.up(x), self.act, getattr(self.down, "takes_quantized_input", False)),
                                 add=add)
        if isinstance(x, PendingNorm):
            if getattr(self.up, "glu_blocked", False):     # batch 1: norm in the gate_up prologue
                return self.down(self.up.glu(x), add=add)
            if self.act == "silu_glu" and type(self.up) is Linear and not x.quant:
                return self.down(self.up.forward_norm(x, glu=True), add=add)   # 16-bit gate_up
            x = x.materialize()
        if getattr(self.up, "glu_blocked", False):
            # W8A8 SwiGLU with 16-blocked gate_up rows: decode-sized batches take the fused
            # GEMV + SwiGLU epilogue (int8 h with per-group scales, or bf16 h that the down
            # projection quantises per group — W8A8Linear.glu); larger ones the blocked
            # activation kernel
            if isinstance(x, QAct) and x.q.dim() == 2 and x.scale.dim() == 1 and self.up.glu_rows_ok(x.q.shape[0]) \
                    and (x.q.shape[0] <= 64 or getattr(self.down, "group_scales_ok", lambda m: False)(x.q.shape[0])):
                return self.down(self.up.glu(x), add=add)
            if isinstance(x, QAct) and x.q.dim() == 2 and x.scale.dim() == 1 and x.q.is_cuda and x.q.is_contiguous() \
                    and _PREFILL_GLU:
                # prefill rows: silu(g) * u in the gate_up GEMM's epilogue (bf16 h, half the bytes
                # of g / u), then the per-token quantisation for the down projection
                h = ops.w8a8_prefill_glu(x.q, x.scale, self.up.w_packed, self.up.w_scale, self.up.bias,
                                      self.up.out_features, self.up.in_features)
                if h is not None:
                    return self.down(QAct(*ops.quant_per_token(h)), add=add)
            return self.down(act_fn(self.up(x), "silu_glu_blocked", True), add=add)
        down_q = getattr(self.down, "takes_quantized_input", False)
        if self.act in ("gelu_tanh", "gelu") and down_q and isinstance(x, QAct) and x.q.dim() == 2 \
                and x.scale.dim() == 1 and getattr(self.up, "geluq_rows_ok", lambda m: False)(x.q.shape[0]) \
                and getattr(self.down, "group_scales_ok", lambda m: False)(x.q.shape[0]):
            # W8A8 GELU MLP (Phi-2, Pythia) at decode rows: up projection + GELU + per-(token, 64)
            # int8 quantisation in one launch, consumed by the down projection's grouped-scale GEMV
            return self.down(self.up.geluq(x, self.act), add=add)
        if self.act == "silu_glu" and type(self.up) is Linear and not down_q and not isinstance(x, QAct) \
                and ops.bf16_gemv_ok(x, self.up.weight, glu=True):
            # bf16 decode: gate_up GEMV with the SwiGLU epilogue (one launch, gemv_bf16.hip)
            return self.down(ops.linear_bf16(x, self.up.weight, self.up.bias, glu=True,
                                             packed=self.up.decode_weight(x, glu=True)), add=add)
        if self.act in ("gelu_tanh", "gelu") and type(self.up) is Linear and not down_q \
                and not isinstance(x, QAct) and ops.bf16_gemv_ok(x, self.up.weight):
            # bf16 decode (Phi-2, Pythia): up-projection GEMV with the GELU epilogue
            return self.down(ops.linear_bf16(x, self.up.weight, self.up.bias, act=self.act,
                                             packed=self.up.decode_weight(x)), add=add)
        if self.act in ("gelu_tanh", "gelu") and hasattr(self.up, "gelu_fused"):
            h = self.up.gelu_fused(x, self.act)               # LLM.int8 batch 1: GELU in the same launch
            if h is not None:
                return self.down(h, add=add)
        h = self.up(x)
        h = act_fn(h, self.act, down_q)
        return self.down(h, add=add)


class DecoderLayer(nn.Module):
    """One decoder block.  ``has_attn`` / ``has_mlp`` False builds half a block (sequential-residual
    architectures only): a pipeline stage boundary may then fall between the attention half
    (norm1 + attention + o) and the MLP half (norm2 + MLP) of a layer.  The hand-off there is the
    residual stream h2 = a + h, exactly the tensor a whole-layer boundary hands over."""

    def __init__(self, cfg: ModelConfig, idx: int, dtype, device, has_attn: bool = True, has_mlp: bool = True):
        super().__init__()
        assert has_attn or has_mlp
        assert (has_attn and has_mlp) or not cfg.parallel_residual, "half layers need a sequential residual"
        self.cfg, self.idx = cfg, idx
        self.has_attn, self.has_mlp = has_attn, has_mlp
        self.norm1 = Norm(cfg.hidden_size, cfg.norm, cfg.norm_eps, dtype, device) if has_attn else None
        self.norm2 = (None if cfg.shared_input_norm or not has_mlp
                      else Norm(cfg.hidden_size, cfg.norm, cfg.norm_eps, dtype, device))
        self.attn = Attention(cfg, idx, dtype, device) if has_attn else None
        self.mlp = MLP(cfg, dtype, device) if has_mlp else None
        if cfg.norm == "rms" and not cfg.parallel_residual:
            # o and down feed an RMSNorm (or the stage exit): bf16 decode GEMVs split K and the norm
            # kernel sums the fp32 slices (quantised replacements set their own split)
            if has_attn:
                self.attn.o.split_k_out = BF16_SPLIT_K
            if has_mlp:
                self.mlp.down.split_k_out = BF16_SPLIT_K

    def _ln_deferred(self, x, qa: bool, qm: bool) -> bool:
        """Parallel-residual 16-bit decode rows whose LayerNorm(s) the qkv / up GEMVs can compute."""
        cfg = self.cfg
        return (not qa and not qm and cfg.norm == "layer" and self.has_attn and self.has_mlp
                and isinstance(x, torch.Tensor) and self.norm1 is not None
                and (cfg.shared_input_norm or self.norm2 is not None)
                and cfg.act in ("gelu_tanh", "gelu") and x.dim() == 2 and ops.gemv_ln_ok(x)
                and _ln_consumer_ok(self.attn.qkv) and _ln_consumer_ok(self.mlp.up)
                and x.dtype == self.norm1.weight.dtype)

    def _ln_deferred_l8(self, x, qa: bool, qm: bool) -> bool:
        """Parallel-residual LLM.int8 rows at batch 1 whose LayerNorm(s) the one-launch qkv / up
        projections can compute."""
        cfg = self.cfg
        ok = lambda m: getattr(m, "takes_pending_x", False) and m.pending_ln_ok()
        return (not qa and not qm and cfg.norm == "layer" and self.has_attn and self.has_mlp
                and isinstance(x, torch.Tensor) and x.dim() == 2 and x.shape[0] == 1 and x.dtype == torch.bfloat16
                and (cfg.shared_input_norm or self.norm2 is not None) and ops.gemv_ln_ok(x)
                and self.norm1.weight.dtype == torch.bfloat16 and ok(self.attn.qkv) and ok(self.mlp.up))

    def _ln_deferred_w8a8(self, x, qa: bool, qm: bool) -> bool:
        """GPT-NeoX W8A8 decode rows whose two LayerNorms the qkv / up GEMVs can compute (Phi shares
        one norm between them, and only one prologue would take it: no gain, not taken)."""
        cfg = self.cfg
        return (qa and qm and cfg.norm == "layer" and not cfg.shared_input_norm and self.has_attn
                and self.has_mlp and self.norm2 is not None and cfg.act in ("gelu_tanh", "gelu")
                and isinstance(x, torch.Tensor) and x.dim() == 2 and x.dtype == torch.bfloat16
                and ops.gemv_ln_ok(x) and self.norm1.weight.dtype == torch.bfloat16
                and getattr(self.attn.qkv, "pending_ln_ok", lambda **k: False)()
                and getattr(self.mlp.up, "pending_ln_ok", lambda **k: False)(geluq=True)
                and getattr(self.mlp.down, "group_scales_ok", lambda m: False)(x.shape[0]))

    def forward(self, x, residual, ctx: AttnCtx):
        cfg = self.cfg
        if not cfg.parallel_residual:
            # <= 4 rows: each norm of a split-K sum runs in the prologue of the W8A8 GEMV after it
            qm = self.mlp.up.takes_quantized_input if self.has_mlp else False
            d2 = getattr(self.mlp.up, "pending_norm_ok", lambda glu=False: False)(glu=True) if self.has_mlp else False
            if self.has_attn:
                qa = self.attn.qkv.takes_quantized_input
                d1 = getattr(self.attn.qkv, "pending_norm_ok", lambda glu=False: False)()
                # 129-256 rows: the qkv projection takes the int8 rows fragment-packed (w8a8_r256)
                n1, h = self.norm1(x, residual, quant=qa, defer=d1, packed_for=self.attn.qkv if qa else None)
                a = self.attn(n1, ctx)
                if not self.has_mlp:
                    return a, h                        # stage exit after the attention half
                n2, h2 = self.norm2(a, h, quant=qm, defer=d2)
            else:
                n2, h2 = self.norm2(x, residual, quant=qm, defer=d2)   # MLP half: x = h2 from the stage before
            return self.mlp(n2), h2
        qa = self.attn.qkv.takes_quantized_input
        qm = self.mlp.up.takes_quantized_input
        if self._ln_deferred_w8a8(x, qa, qm):
            # W8A8 decode at batch 1 (GPT-NeoX): LayerNorm + int8 quant in the qkv / up GEMV prologues
            n1, n2, h = self.norm1, self.norm2, torch.empty_like(x)
            pa = PendingLN(x, residual, n1.weight, n1.bias, n1.eps, h, None, True)
            pm = PendingLN(x, residual, n2.weight, n2.bias, n2.eps, h, None, True)
            return self.mlp(pm, add=self.attn(pa, ctx)), h
        if self._ln_deferred_l8(x, qa, qm):
            # LLM.int8 at batch 1: the LayerNorm(s) inside the one-launch qkv / up projections
            n1, h = self.norm1, torch.empty_like(x)
            if cfg.shared_input_norm:                  # phi: qkv also writes the normalised row for up
                y = torch.empty_like(x)
                pa = PendingLN(x, residual, n1.weight, n1.bias, n1.eps, h, y)
                pm = y
            else:
                n2 = self.norm2
                pa = PendingLN(x, residual, n1.weight, n1.bias, n1.eps, h)
                pm = PendingLN(x, residual, n2.weight, n2.bias, n2.eps, h)
            return self.mlp(pm, add=self.attn(pa, ctx)), h
        if self._ln_deferred(x, qa, qm):
            # 16-bit decode at batch 1: each consumer computes the LayerNorm in its GEMV prologue
            n1, h = self.norm1, torch.empty_like(x)
            if cfg.shared_input_norm:
                # phi: the qkv GEMV computes the norm and also writes it for the up projection
                # (a second prologue would cost more than it saves: 1.726 -> 1.775 ms per step)
                y = torch.empty_like(x)
                pa = PendingLN(x, residual, n1.weight, n1.bias, n1.eps, h, y)
                pm = y
            else:                                              # gpt_neox: norm2 of h = x + residual
                n2 = self.norm2
                pa = PendingLN(x, residual, n1.weight, n1.bias, n1.eps, h)
                pm = PendingLN(x, residual, n2.weight, n2.bias, n2.eps, h)
            return self.mlp(pm, add=self.attn(pa, ctx)), h
        if cfg.shared_input_norm:                      # phi
            n, h = self.norm1(x, residual, quant=qa and qm)
            if qa != qm:                               # mixed modes: feed each consumer its form
                n, h = self.norm1(x, residual, quant=False)
                na, nm = quant_if(n, self.attn.qkv), quant_if(n, self.mlp.up)
            else:
                na = nm = n
            # attn + mlp: the sum is taken in the down projection's epilogue (one launch fewer)
            return self.mlp(nm, add=self.attn(na, ctx)), h
        n1, h = self.norm1(x, residual, quant=qa)      # gpt_neox
        n2, _ = self.norm2(h, None, quant=qm)
        return self.mlp(n2, add=self.attn(n1, ctx)), h


def _ln_consumer_ok(lin) -> bool:
    return type(lin) is Linear and lin.pending_ln_ok()


class DecoderLM(nn.Module):
    """A (possibly partial) causal LM.  ``first``/``last`` select the layers this instance
    owns; embedding and head are present only on the first / last stage."""

    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None, first: int = 0,
                 last: Optional[int] = None, split_first: bool = False, split_last: bool = False):
        """``split_first``: layer ``first`` holds only its MLP half; ``split_last``: layer
        ``last - 1`` only its attention half (sub-layer pipeline boundaries, see ``from_units``)."""
        super().__init__()
        self.cfg = cfg
        self.dtype = dtype
        self.first = first
        self.last = cfg.num_layers if last is None else last
        assert self.last > first or not (split_first or split_last)
        assert not (split_first and split_last and self.last - first == 1), "an empty half-layer stage"
        self.split_first, self.split_last = bool(split_first), bool(split_last)
        self.units = (2 * first + self.split_first, 2 * self.last - self.split_last)
        self.kv_first = first + self.split_first           # first layer with attention (KV cache)
        self.has_embed = first == 0 and not self.split_first
        self.has_head = self.last == cfg.num_layers and not self.split_last
        if self.has_embed:
            self.embed = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden_size, dtype=dtype, device=device),
                                      requires_grad=False)
            self.pos_embed = (nn.Parameter(torch.empty(cfg.max_position_embeddings, cfg.hidden_size, dtype=dtype,
                                                       device=device), requires_grad=False)
                              if cfg.pos_emb == "learned" else None)
        self.layers = nn.ModuleList([
            DecoderLayer(cfg, i, dtype, device, has_attn=not (self.split_first and i == first),
                         has_mlp=not (self.split_last and i == self.last - 1))
            for i in range(self.first, self.last)])
        if self.has_head:
            self.final_norm = Norm(cfg.hidden_size, cfg.norm, cfg.norm_eps, dtype, device)
            if cfg.tie_word_embeddings and self.has_embed:
                self.lm_head = None
            else:
                self.lm_head = Linear(cfg.hidden_size, cfg.vocab_size, cfg.lm_head_bias, dtype, device)
        self._rope = None

    @classmethod
    def from_units(cls, cfg: ModelConfig, ua: int, ub: int, **kw) -> "DecoderLM":
        """Stage of half-layer units [ua, ub): unit 2 i is layer i's attention half, 2 i + 1 its
        MLP half (ub == 2 * num_layers: through the head)."""
        assert 0 <= ua < ub <= 2 * cfg.num_layers or ua == ub == 2 * cfg.num_layers
        return cls(cfg, first=ua // 2, last=(ub + 1) // 2, split_first=ua % 2 == 1, split_last=ub % 2 == 1, **kw)

    # ------------------------------------------------------------------ helpers
    @property
    def device(self):
        return next(self.parameters()).device

    def rope_table(self, device=None) -> Optional[torch.Tensor]:
        cfg = self.cfg
        if cfg.pos_emb != "rope":
            return None
        device = device or self.device
        if self._rope is None or self._rope.device != torch.device(device):
            self._rope = ops.rope_tables(cfg.rotary_dim, cfg.max_position_embeddings, cfg.rope_theta,
                                         cfg.rope_scaling, device=device)
        return self._rope

    def head_weight(self) -> torch.Tensor:
        return self.embed if self.lm_head is None else self.lm_head.weight

    def _first_norm_deferred(self, rows: int) -> bool:
        """Whether the first layer's RMSNorm can run in its qkv GEMV's prologue at ``rows`` decode
        rows: the embedding is then handed over as one fp32 split-K slice (no residual), which
        saves the norm launch (batch 1)."""
        if rows > ops.NORM_FUSE_MAX_ROWS or self.pos_embed is not None or self.cfg.parallel_residual:
            return False
        first = self.layers[0] if len(self.layers) else None
        if first is None or not first.has_attn or first.norm1 is None or first.norm1.kind != "rms":
            return False
        qkv = first.attn.qkv
        ok = getattr(qkv, "pending_norm_ok", lambda glu=False: False)()
        return ok is not False and ok != "x" and bool(ok)     # ("x": a consumer of the bf16 row itself)

    def embed_tokens(self, ids: torch.Tensor, start_pos: torch.Tensor, decode: bool = False):
        """ids [B, T] -> hidden [B*T, H] (``decode`` at batch 1 with a deferrable first norm: a
        PartialSum [1, B*T, H] of fp32 rows, which the first norm sums like a split-K slice)."""
        B, T = ids.shape
        if decode and ops.gpu_path(self.embed) and self._first_norm_deferred(B * T):
            xf = ops.embedding(ids.reshape(-1), self.embed, out_f32=True)
            if ops.gemv_norm_ok(xf.view(1, B * T, -1)):
                return PartialSum(xf.view(1, B * T, -1), self.embed.dtype)
        x = ops.embedding(ids.reshape(-1), self.embed)
        if self.pos_embed is not None:
            pos = (start_pos.long()[:, None] + torch.arange(T, device=ids.device)[None]).reshape(-1)
            x = x + self.pos_embed[pos]
        return x

    # ------------------------------------------------------------------ forward
    def forward_layers(self, x: torch.Tensor, ctx: AttnCtx, residual: Optional[torch.Tensor] = None):
        if tracing.TRACE:                      # roctx range per layer (rocprofv3 --marker-trace)
            for layer in self.layers:
                with tracing.trace_range(f"{ctx.mode}.layer{layer.idx}"):
                    x, residual = layer(x, residual, ctx)
            return x, residual
        for layer in self.layers:
            x, residual = layer(x, residual, ctx)
        return x, residual

    def head(self, x: torch.Tensor, residual: Optional[torch.Tensor], ctx: AttnCtx,
             logits: str = "last") -> torch.Tensor:
        """Final norm + LM head. logits: "last" (one row per sequence) or "all"; "hidden": the
        final-normed last rows only, for an LM head split by vocabulary over pipeline ranks
        (parallel/vocab_head.py)."""
        last = logits in ("last", "hidden")
        if isinstance(x, PartialSum) and last and ctx.T > 1:
            x = x.materialize()
        if last and ctx.T > 1:
            idx = ctx.last_rows(x.device)
            x = x.index_select(0, idx)
            residual = residual.index_select(0, idx) if residual is not None else None
        qh = getattr(self.lm_head, "takes_quantized_input", False) and logits != "hidden"   # int8 LM head
        h, _ = self.final_norm(x, residual, quant=qh)
        if logits == "hidden":
            return h
        return self.lm_head(h) if self.lm_head is not None else self._tied_head(h)

    def _tied_head(self, h: torch.Tensor) -> torch.Tensor:
        """LM head on the embedding matrix (tied models): decode-sized rows take the bf16 GEMV on a
        fragment-packed copy of the embedding, built on the first decode call and kept (Llama-3.2-1B
        batch 1: hipBLASLt's small-M kernel ran the 525 MB head at 4.6 TB/s, 113 us per token)."""
        if not ops.bf16_gemv_ok(h, self.embed):
            return torch.nn.functional.linear(h, self.embed)
        wp, ver = getattr(self, "_embed_wp", None), self.embed._version
        if wp is None or getattr(self, "_embed_wp_ver", -1) != ver or wp.device != self.embed.device:
            wp = self._embed_wp = ops.pack_bf16_weight(self.embed.detach())
            self._embed_wp_ver = ver
        return ops.linear_bf16(h, self.embed, None, packed=wp)

    def _b1_engine(self, ctx: AttnCtx):
        """The batch-1 persistent decode engine for this step, or None (not eligible / not batch 1)."""
        if ctx.mode != "decode" or ctx.B != 1 or ctx.T != 1 or ctx.attn_hook is not None or not self.has_embed:
            return None
        kv = ctx.kv
        if hasattr(kv, "cache"):                         # KVView: row 0 of a cache
            if kv.r0 != 0:
                return None
            kv = kv.cache
        if not hasattr(kv, "k") or not ops.gpu_path(self.embed):
            return None
        from ..engine import b1_engine
        return b1_engine.engine_for(self, kv)

    def forward(self, ids: Optional[torch.Tensor], ctx: AttnCtx, hidden: Optional[torch.Tensor] = None,
                logits: str = "last"):
        """First stage: ids [B, T]; later stages: hidden [B*T, H] from the previous stage.
        Returns logits on the last stage, otherwise the hidden handed to the next stage."""
        if ctx.b1 and ids is not None:
            eng = self._b1_engine(ctx)
            if eng is not None:
                # every layer in one launch (embedding -> engine -> final norm + LM head)
                h = eng.run(ops.embedding(ids.reshape(-1), self.embed), ctx.start_pos)
                return self.head(h, None, ctx, logits)
        x = self.embed_tokens(ids, ctx.start_pos, decode=ctx.mode == "decode") if self.has_embed else hidden
        x, residual = self.forward_layers(x, ctx, None)
        if self.has_head:
            return self.head(x, residual, ctx, logits)
        if isinstance(x, PartialSum):
            x = x.materialize()
        return x + residual if residual is not None else x


# --------------------------------------------------------------------------- initialisation


@torch.no_grad()
def init_random_(model: DecoderLM, seed: int = 0, std: float = 0.02) -> DecoderLM:
    """Random-init weights (HF-style N(0, 0.02), norms = 1, biases = 0), generated on the
    model's device.  Used for benchmarks and tests (no checkpoints are downloaded)."""
    for name, p in global_named_parameters(model):
        if name.endswith("norm1.weight") or name.endswith("norm2.weight") or name.endswith("final_norm.weight"):
            p.fill_(1.0)
        elif name.endswith("bias"):
            p.zero_()
        else:
            # seeded by the GLOBAL parameter name: a pipeline stage holding layers [a, b) gets
            # bit-identical weights to the same layers of the unsplit model
            if name == "lm_head.weight" and model.cfg.tie_word_embeddings:
                name = "embed"  # head-only stage of a tied model: same values as the embedding
            g = torch.Generator(device=p.device).manual_seed((seed * 1000003 + zlib.crc32(name.encode())) % (2 ** 63))
            p.copy_(torch.randn(p.shape, generator=g, device=p.device, dtype=torch.float32).mul_(std).to(p.dtype))
    return model


def random_head_weight(cfg: ModelConfig, seed: int = 0, dtype=torch.bfloat16, device=None,
                       std: float = 0.02) -> torch.Tensor:
    """The LM-head weight [V, H] ``init_random_`` gives a model holding the head (the embedding of a
    tied model), built on a rank that holds no head (a vocab shard of it, parallel/vocab_head.py)."""
    name = "embed" if cfg.tie_word_embeddings else "lm_head.weight"
    g = torch.Generator(device=device).manual_seed((seed * 1000003 + zlib.crc32(name.encode())) % (2 ** 63))
    return torch.randn((cfg.vocab_size, cfg.hidden_size), generator=g, device=device,
                       dtype=torch.float32).mul_(std).to(dtype)


def global_named_parameters(model: DecoderLM):
    """named_parameters() with layer indices rewritten to global layer numbers."""
    for name, p in model.named_parameters():
        if name.startswith("layers."):
            _, local, rest = name.split(".", 2)
            name = f"layers.{model.layers[int(local)].idx}.{rest}"
        yield name, p


def build_model(cfg: ModelConfig, dtype=torch.bfloat16, device=None, first: int = 0, last: Optional[int] = None,
                seed: Optional[int] = 0, units: Optional[tuple] = None) -> DecoderLM:
    """``units=(ua, ub)``: a sub-layer stage (``DecoderLM.from_units``) instead of layers [first, last)."""
    if units is not None:
        m = DecoderLM.from_units(cfg, units[0], units[1], dtype=dtype, device=device).eval()
    else:
        m = DecoderLM(cfg, dtype=dtype, device=device, first=first, last=last).eval()
    if seed is not None:
        init_random_(m, seed)
    return m

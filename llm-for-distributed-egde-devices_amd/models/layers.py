"""Building blocks shared by every decoder family.

``Linear`` is the bf16 projection (decode rows: ``gemv_bf16.hip`` up to 16, the bf16 ring GEMM
up to 256; otherwise hipBLASLt through ``F.linear`` — ``ops.linear_bf16``);
quantised replacements live in ``edgellm.quant`` and expose the same interface:

    forward(x)                 -> y     x is bf16, or a QAct (int8 + per-token scale) when
    takes_quantized_input      -> bool  the layer wants its producer to emit int8 directly
                                        (the W8A8 fusion: norm/activation kernels quantise in
                                        their epilogue, so no bf16 activation round trip).
"""
from __future__ import annotations

from typing import NamedTuple, Optional

import torch
import torch.nn as nn

from .. import ops


class QAct(NamedTuple):
    """Per-token symmetric INT8 activation: x ~= q * scale[:, None].  ``packed``: q is the [M, K]
    view of a fragment-packed [256, K] buffer (the 256-row decode GEMM's operand layout, written by
    the norm kernel: ops.rms_norm_quant(..., packed=True)); only ``W8A8Linear`` reads it."""
    q: torch.Tensor
    scale: torch.Tensor
    packed: bool = False


class PartialSum(NamedTuple):
    """Split-K output of a decode projection: fp32 slices [S, M, N] whose in-order sum, rounded
    to ``dtype`` (the model's 16-bit type), is the projection's output.  RMSNorm consumes it
    directly (one kernel adds the slices); anything else calls ``materialize()``."""
    parts: torch.Tensor
    dtype: torch.dtype = torch.bfloat16

    def materialize(self) -> torch.Tensor:
        acc = self.parts[0].clone()
        for s in range(1, self.parts.shape[0]):      # same order as the norm kernel
            acc += self.parts[s]
        return acc.to(self.dtype)


class PendingNorm(NamedTuple):
    """RMSNorm (+ per-token int8 quant when ``quant``) of a decode split-K PartialSum (+ residual,
    M <= 4 rows), deferred into the prologue of the GEMV that consumes it (W8A8: ops.w8a8_gemv_norm;
    16-bit: ops.gemv_bf16_norm): one launch fewer per norm.  ``h`` is the residual-stream output
    [M, H], written by that GEMV.  ``materialize()`` runs the norm kernel instead (into ``h``) for a
    consumer that cannot take it."""
    parts: torch.Tensor
    residual: torch.Tensor
    weight: torch.Tensor
    eps: float
    h: torch.Tensor
    quant: bool = True

    def materialize(self):
        y, s, r = ops.rms_norm_parts(self.parts, self.residual, self.weight, self.eps, self.quant)
        self.h.copy_(r.view_as(self.h))
        return QAct(y, s) if self.quant else y


class PendingLN(NamedTuple):
    """LayerNorm of 16-bit decode rows x (+ residual, M <= 4), deferred into the prologue of the
    16-bit GEMV(s) that consume it (ops.gemv_bf16_ln; parallel-residual blocks, where the qkv and
    the MLP up projection both read a norm of the same rows): no norm launch.  ``h`` = x + residual,
    written by the consumer (every consumer writes the same bits); ``y`` (optional): the consumer
    also writes the normalised rows there, for a second consumer that reads them as a plain input.
    ``materialize()`` runs the norm kernel instead."""
    x: torch.Tensor
    residual: Optional[torch.Tensor]
    weight: torch.Tensor
    bias: Optional[torch.Tensor]
    eps: float
    h: torch.Tensor
    y: Optional[torch.Tensor] = None
    quant: bool = False              # the consumers are W8A8: int8 rows per token (QAct)
    rms: bool = False                # RMSNorm (no bias) instead of LayerNorm (LLM.int8 consumers only)

    def materialize(self):
        if self.rms:
            y, r = ops.rms_norm(self.x, self.weight, self.eps, self.residual)
            self.h.copy_(r.view_as(self.h))
            if self.y is not None:
                self.y.copy_(y.view_as(self.y))
            return y
        if self.quant:
            q, s, r = ops.layer_norm_quant(self.x, self.weight, self.bias, self.eps, self.residual)
            self.h.copy_(r.view_as(self.h))
            return QAct(q, s)
        y, r = ops.layer_norm(self.x, self.weight, self.bias, self.eps, self.residual)
        self.h.copy_(r.view_as(self.h))
        if self.y is not None:
            self.y.copy_(y.view_as(self.y))
        return y


class GroupQuantBF16(NamedTuple):
    """bf16 activation that a W8A8 consumer quantises per (token, 64 columns) on the fly."""
    x: torch.Tensor


class Linear(nn.Module):
    takes_quantized_input = False
    split_k_out = 0     # > 0: decode calls return split-K fp32 partials (PartialSum) for the next norm

    def __init__(self, in_features: int, out_features: int, bias: bool = False, dtype=torch.bfloat16,
                 device=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=dtype, device=device),
                                   requires_grad=False)
        self.bias = (nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device), requires_grad=False)
                     if bias else None)

    def pending_norm_ok(self, glu: bool = False) -> bool:
        """Whether this 16-bit projection takes a PendingNorm (its decode GEMV computes the RMSNorm
        in its prologue, gemv_bf16.hip); glu: as the [gate | up] projection of a SwiGLU MLP."""
        w = self.weight
        return (w.is_cuda and w.dtype in (torch.bfloat16, torch.float16) and ops.available()
                and self.in_features in (2048, 4096) and self.out_features % (32 if glu else 16) == 0
                and not self.split_k_out and ops.gpu_path(w))

    def packed_weight(self) -> torch.Tensor:
        """The fragment-packed decode copy of the weight (``decode_weight`` without a sample input)."""
        wp, ver = getattr(self, "_wp", None), self.weight._version
        if wp is None or getattr(self, "_wp_ver", -1) != ver or wp.device != self.weight.device:
            wp = self._wp = ops.pack_bf16_weight(self.weight.detach())
            self._wp_ver = ver
        return wp

    def forward_norm(self, x: "PendingNorm", glu: bool = False):
        """The decode GEMV over a PendingNorm (RMSNorm in the prologue); glu: silu(gate) * up."""
        y = None
        if self.pending_norm_ok(glu) and x.parts.dtype == torch.float32:
            y = ops.gemv_bf16_norm(x.parts, x.residual, x.weight, x.eps, x.h, self.packed_weight(), self.bias,
                                   self.out_features, glu=glu)
        if y is not None:
            return y
        xm = x.materialize()
        if glu:
            return ops.linear_bf16(xm, self.weight, self.bias, glu=True, packed=self.decode_weight(xm, glu=True))
        return self.forward(xm)

    def pending_ln_ok(self) -> bool:
        """Whether this 16-bit projection's decode GEMV can compute a LayerNorm in its prologue."""
        w = self.weight
        return (w.is_cuda and w.dtype in (torch.bfloat16, torch.float16) and ops.available()
                and self.in_features <= 4096 and self.in_features % 64 == 0 and self.out_features % 16 == 0
                and not self.split_k_out and ops.gpu_path(w))

    def forward_ln(self, x: "PendingLN", act: Optional[str] = None):
        """The decode GEMV over a PendingLN (LayerNorm in the prologue); act: its GELU epilogue."""
        y = None
        if self.pending_ln_ok() and x.x.dtype == self.weight.dtype and not x.rms:
            y = ops.gemv_bf16_ln(x.x, x.residual, x.weight, x.bias, x.eps, x.h, self.packed_weight(), self.bias,
                                 self.out_features, act, y_out=x.y)
        if y is not None:
            return y
        xm = x.materialize()
        if act is not None:
            return ops.linear_bf16(xm, self.weight, self.bias, act=act, packed=self.decode_weight(xm))
        return self.forward(xm)

    def forward(self, x, add=None):
        """``add``: the other branch of a parallel-residual block, added to the output (in the
        decode GEMV's epilogue where that kernel runs)."""
        if isinstance(x, PendingLN):
            assert add is None, "a PendingLN consumer has no addend"
            return self.forward_ln(x)
        if isinstance(x, PendingNorm):
            assert add is None, "a PendingNorm consumer has no addend"
            return self.forward_norm(x)
        if isinstance(x, QAct):
            x = (x.q.float() * x.scale[..., None]).to(self.weight.dtype)
        wp = self.decode_weight(x)
        if self.split_k_out and wp is not None and add is None:
            K = x.shape[-1]
            if ops.bf16_decode_mode(x, self.weight, split=True) == 2:
                # 17-256 rows: the ring GEMM's split-K slices (the launcher picks S for the shape)
                S = int(ops.ext().bf16_ring_splits(self.out_features, K))
                if S > 1:
                    return PartialSum(ops.ext().gemm_bf16_ring(x.reshape(-1, K), wp, self.bias,
                                                               self.out_features, 3, S))
            elif K // 64 >= self.split_k_out:
                return PartialSum(ops.ext().gemv_bf16_splitk(x.reshape(-1, K), wp, self.bias,
                                                             self.out_features, self.split_k_out), x.dtype)
        return ops.linear_bf16(x, self.weight, self.bias, packed=wp,
                               add=None if add is None else add.reshape(*x.shape[:-1], self.out_features))

    def decode_weight(self, x, glu: bool = False) -> "Optional[torch.Tensor]":
        """Fragment-packed copy of the weight for the decode GEMV / ring GEMM, built on the first
        decode-sized call (before any graph capture) and kept; None when not applicable."""
        if not ops.bf16_decode_mode(x, self.weight, glu=glu, split=bool(self.split_k_out)):
            return None
        wp, ver = getattr(self, "_wp", None), self.weight._version   # in-place weight edits repack
        if wp is None or getattr(self, "_wp_ver", -1) != ver or wp.device != self.weight.device:
            wp = self._wp = ops.pack_bf16_weight(self.weight.detach())
            self._wp_ver = ver
        return wp

    def extra_repr(self):
        return f"{self.in_features}->{self.out_features}, bias={self.bias is not None}, {str(self.weight.dtype)[6:]}"


class Norm(nn.Module):
    """RMSNorm or LayerNorm with fused residual add and optional fused INT8 quant epilogue."""

    def __init__(self, hidden: int, kind: str, eps: float, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.kind, self.eps = kind, eps
        self.weight = nn.Parameter(torch.ones(hidden, dtype=dtype, device=device), requires_grad=False)
        self.bias = (nn.Parameter(torch.zeros(hidden, dtype=dtype, device=device), requires_grad=False)
                     if kind == "layer" else None)

    def forward(self, x, residual=None, quant: bool = False, defer: bool = False, packed_for=None):
        """Returns (y, residual_out) where residual_out = x + residual; y is a QAct when quant.
        ``x`` may be a PartialSum (split-K projection output), summed inside the norm kernel.
        ``defer`` (the consumer is a W8A8 GEMV that takes it): at <= 4 rows, y is a PendingNorm that
        the consumer's kernel computes, and residual_out is the buffer it fills.
        ``packed_for`` (the consumer projection): when it takes a fragment-packed activation at these
        rows (``W8A8Linear.takes_packed``), the int8 rows are written packed (QAct.packed)."""
        if quant and self.kind == "rms" and packed_for is not None:
            M = (x.parts.shape[1] if isinstance(x, PartialSum) else x.numel() // x.shape[-1])
            if getattr(packed_for, "takes_packed", lambda m: False)(M):
                if isinstance(x, PartialSum):
                    y, s, r = ops.rms_norm_parts(x.parts, residual, self.weight, self.eps, True, packed=True)
                else:
                    y, s, r = ops.rms_norm_quant(x, self.weight, self.eps, residual, packed=True)
                return QAct(y, s, True), r
        if defer == "x" and not quant and isinstance(x, torch.Tensor) and self.kind == "rms" and x.dim() == 2 \
                and x.shape[0] == 1 and ops.gemv_ln_ok(x) and x.dtype == torch.bfloat16:
            # an LLM.int8 consumer at batch 1: the norm of the bf16 row x (+ residual) in its prologue
            h = torch.empty_like(x)
            return PendingLN(x, residual, self.weight, None, self.eps, h, rms=True), h
        if defer and defer != "x" and isinstance(x, PartialSum) and self.kind == "rms" and ops.gemv_norm_ok(x.parts) \
                and (quant or self.weight.dtype == x.dtype):
            # residual None: a stage's first norm, over the embedding as one fp32 slice; a 16-bit
            # consumer (not quant) takes the normalised rows in its own dtype
            h = torch.empty(x.parts.shape[1], x.parts.shape[2], dtype=self.weight.dtype, device=x.parts.device)
            return PendingNorm(x.parts, residual, self.weight, self.eps, h, quant), h
        if isinstance(x, PartialSum):
            if self.kind == "rms" and x.parts.is_cuda and ops.gpu_path(x.parts):
                y, s, r = ops.rms_norm_parts(x.parts, residual, self.weight, self.eps, quant)
                return (QAct(y, s) if quant else y), r
            x = x.materialize()
        if self.kind == "rms":
            if quant:
                q, s, r = ops.rms_norm_quant(x, self.weight, self.eps, residual)
                return QAct(q, s), r
            return ops.rms_norm(x, self.weight, self.eps, residual)
        if quant:
            q, s, r = ops.layer_norm_quant(x, self.weight, self.bias, self.eps, residual)
            return QAct(q, s), r
        return ops.layer_norm(x, self.weight, self.bias, self.eps, residual)


def act_fn(x, act: str, quant: bool):
    if quant:
        q, s = ops.activation_quant(x, act)
        return QAct(q, s)
    return ops.activation(x, act)


def quant_if(x: torch.Tensor, layer) -> object:
    """Quantise a bf16 activation when the consumer wants INT8 input."""
    if getattr(layer, "takes_quantized_input", False):
        q, s = ops.quant_per_token(x)
        return QAct(q, s)
    return x

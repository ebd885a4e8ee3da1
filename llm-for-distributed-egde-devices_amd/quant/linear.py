"""Quantised linear layers (drop-in for ``models.layers.Linear``).

* ``W8A8Linear``   — SmoothQuant-style W8A8: int8 weights with per-output-channel scales,
  int8 activations with per-token scales produced by the *previous* kernel's epilogue (fused
  norm/activation quant), INT8 MFMA GEMM with fused dequant (+bias) epilogue.  The north-star
  quantised path (new capability: the reference has no SmoothQuant code).
* ``LLMInt8Linear`` — compatibility mode for the reference's bitsandbytes ``LLM.int8()``
  (``BitsAndBytesConfig(load_in_8bit=True)``, Code/Quantised Models/models_quant_updated.py:30-32):
  weights int8 with per-row absmax ``SCB``; activation columns with any |x| > threshold (6.0)
  are "outliers" computed in bf16 against the dequantised weight columns, the rest goes
  through the same INT8 GEMM with per-token scales.
* ``CPUDynamicLinear`` — the reference's CPU edge path, ``torch.quantization.quantize_dynamic``
  on nn.Linear with qint8 (Code/C-DAC Server/try.py:198-206).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from ..ops import _ref
from ..models.layers import GroupQuantBF16, Linear, PartialSum, PendingLN, PendingNorm, QAct

# Decode MLP policy (A/B on MI355X, Llama-2-7B, profiles/bench_ops_r1_gemv16.json): the gate_up
# GEMV quantises silu(g) * u in its own epilogue (8 tiles = 64 features per workgroup) for every
# decode batch — 21.7 us vs 26.5 us for bf16 h + the group-quant kernel at 16 rows, and ahead at
# 1, 33 and 64 rows too.  EDGELLM_GLU_QUANT_MIN_ROWS raises the threshold (A/B runs).
GLU_QUANT_MIN_ROWS = int(os.environ.get("EDGELLM_GLU_QUANT_MIN_ROWS", "1"))


def glu_quant_rows(m: int) -> bool:
    return m >= GLU_QUANT_MIN_ROWS


def quantize_weight_per_channel(w: torch.Tensor):
    """Symmetric per-output-row int8: returns (q [N,K] int8, scale [N] f32)."""
    wf = w.float()
    amax = wf.abs().amax(1).clamp_min(1e-8)
    scale = amax / 127.0
    q = torch.round(wf / scale[:, None]).clamp_(-127, 127).to(torch.int8)
    return q, scale


class W8A8Linear(nn.Module):
    takes_quantized_input = True
    graph_safe = True

    def __init__(self, in_features: int, out_features: int, bias: bool, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        kt, nt = (in_features + 63) // 64, (out_features + 15) // 16
        self.register_buffer("w_packed", torch.zeros(nt * kt * 1024, dtype=torch.int8, device=device))
        self.register_buffer("w_scale", torch.ones(out_features, dtype=torch.float32, device=device))
        self.register_buffer("bias", torch.zeros(out_features, dtype=dtype, device=device) if bias else None)
        self._w_cpu = None
        self.out_dtype = dtype
        self.glu_blocked = False      # rows stored 16-blocked [gate(16) | up(16)] (fused decode GLU)
        self.split_k_out = 0          # > 0: decode output as split-K PartialSum (consumer is an RMSNorm)

    @classmethod
    @torch.no_grad()
    def from_float(cls, lin: Linear, smooth: Optional[torch.Tensor] = None) -> "W8A8Linear":
        """smooth[k] multiplies input column k of W (the activation is divided by it upstream)."""
        w = lin.weight.float()
        if smooth is not None:
            w = w * smooth.float()[None, :].to(w.device)
        q, s = quantize_weight_per_channel(w)
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, device=w.device, dtype=lin.weight.dtype)
        m.load_int8(q, s, lin.bias)
        return m

    @torch.no_grad()
    def load_int8(self, q: torch.Tensor, scale: torch.Tensor, bias: Optional[torch.Tensor] = None):
        self.w_packed.copy_(ops.pack_int8_weight(q.to(self.w_packed.device)))
        self.w_scale.copy_(scale.float())
        if bias is not None:
            self.bias.copy_(bias)
        self._w_cpu = None

    def int8_weight(self) -> torch.Tensor:
        return ops.unpack_int8_weight(self.w_packed, self.out_features, self.in_features)

    def dequant_weight(self) -> torch.Tensor:
        return self.int8_weight().float() * self.w_scale[:, None]

    @torch.no_grad()
    def block_glu_(self) -> "W8A8Linear":
        """Re-pack a [gate | up] projection 16-blocked so one 2-tile GEMV workgroup holds both
        halves of 16 features (the fused SwiGLU epilogue, ops.w8a8_glu).  Outputs of ``forward``
        are then in blocked order (activation ``silu_glu_blocked``)."""
        if not self.glu_blocked:
            q, sc, b = self.canonical()
            self.load_int8(_ref.block_glu_rows(q), _ref.block_glu_rows(sc),
                           _ref.block_glu_rows(b) if b is not None else None)
            self.glu_blocked = True
        return self

    def canonical(self):
        """(int8 weight, w_scale, bias) in the un-blocked [gate | up] row order (checkpoints)."""
        q, sc, b = self.int8_weight(), self.w_scale, self.bias
        if self.glu_blocked:
            q, sc = _ref.unblock_glu_rows(q), _ref.unblock_glu_rows(sc)
            b = _ref.unblock_glu_rows(b) if b is not None else None
        return q, sc, b

    def _wref(self, x):
        if x.is_cuda:
            return None
        if self._w_cpu is None:
            self._w_cpu = self.int8_weight()
        return self._w_cpu

    def takes_packed(self, M: int) -> bool:
        """Whether this projection takes a fragment-packed activation at M rows (the 256-row decode
        GEMM on the GPU: ops.r256_ok; not split-K outputs, not the GLU projection)."""
        return (self.w_packed.is_cuda and ops.gpu_path(self.w_packed) and not self.split_k_out and
                not self.glu_blocked and ops.r256_ok(M, self.out_features, self.in_features))

    def forward(self, x, add=None):
        """``add``: the other branch of a parallel-residual block, added to the output (in the
        decode GEMV's epilogue at <= 64 rows)."""
        if isinstance(x, QAct) and x.packed:
            K, N = self.in_features, self.out_features
            M = x.q.shape[0]
            y = ops.w8a8_r256(x.q, x.scale, self.w_packed, self.w_scale, self.bias, N, K) if add is None else None
            if y is not None:
                return y
            x = QAct(ops.unpack_a(x.q, M, K), x.scale)      # (a consumer that cannot take it)
        if isinstance(x, PendingLN):                  # batch 1: the LayerNorm in this GEMV's prologue
            y = None
            if add is None and not self.split_k_out:
                y = ops.w8a8_gemv_ln(x.x, x.residual, x.weight, x.bias, x.eps, x.h, self.w_packed, self.w_scale,
                                     self.bias, self.out_features, self.in_features)
            if y is not None:
                return y
            x = x.materialize()
        if isinstance(x, PendingNorm):                # batch 1: the norm runs in this GEMV's prologue
            y = None
            if add is None and not self.split_k_out:
                y = ops.w8a8_gemv_norm(x.parts, x.residual, x.weight, x.eps, x.h, self.w_packed, self.w_scale,
                                       self.bias, self.out_features, self.in_features)
            if y is not None:
                return y
            x = x.materialize()
        if isinstance(x, GroupQuantBF16):             # decode: per-(token, 64) int8 input
            x = QAct(*ops.quant_per_group(x.x.reshape(-1, self.in_features)))
        if not isinstance(x, QAct):
            x = QAct(*ops.quant_per_token(x))
        K, N = self.in_features, self.out_features
        shp = x.q.shape[:-1]
        scale = x.scale if x.scale.dim() == 2 and x.q.dim() == 2 else x.scale.reshape(-1)
        M = x.q.numel() // K
        if add is not None:
            out = ops.w8a8_linear(x.q.reshape(-1, K), scale, self.w_packed, self.w_scale, self.bias, N, K,
                                  w_ref=self._wref(x.q), out_dtype=self.out_dtype, add=add.reshape(M, N))
            return out.view(*shp, N)
        if self.split_k_out and x.q.is_cuda and ops.gpu_path(x.q) and K % 64 == 0 and 0 < M and \
                ops.decode_rows_ok(M, K, 4 if M > 64 else 1):
            return PartialSum(ops.w8a8_linear_splitk(x.q.reshape(-1, K), scale, self.w_packed, self.w_scale,
                                                     self.bias, N, K,
                                                     self.split_k_out if self.split_k_out > 1 and M <= 64 else 0))
        out = ops.w8a8_linear(x.q.reshape(-1, K), scale, self.w_packed, self.w_scale, self.bias,
                              N, K, w_ref=self._wref(x.q), out_dtype=self.out_dtype)
        return out.view(*shp, N)

    def group_scales_ok(self, M: int) -> bool:
        """Whether this projection consumes per-(token, 64) activation scales at M rows."""
        K = self.in_features
        return ops.group_scale_rows_ok(M) and \
            (ops.decode_rows_ok(M, K) or (bool(self.split_k_out) and ops.decode_rows_ok(M, K, 4)))

    def glu_rows_ok(self, M: int) -> bool:
        """Whether the fused gate_up + SwiGLU kernel takes M rows (65-128: quantising form only)."""
        return M <= 64 or (self.out_features % 128 == 0 and ops.decode_rows_ok(M, self.in_features)
                           and ops.group_scale_rows_ok(M))

    def pending_norm_ok(self, glu: bool = False) -> bool:
        """Whether this projection takes a PendingNorm (batch-1 RMSNorm in its GEMV prologue)."""
        if glu:
            return self.glu_blocked and self.out_features % 128 == 0
        return not self.split_k_out and not self.glu_blocked

    def glu(self, x: QAct):
        """Fused gate_up -> silu(g) * u (blocked layout, M <= 64) for the down projection: int8
        quantised per (token, 64 features) in the same kernel (``QAct`` with 2-D scales) when
        ``glu_quant_rows(M)``, else bf16 h that the down projection quantises per group.  A
        PendingNorm input (batch 1) is normalised in the same kernel's prologue."""
        K, N = self.in_features, self.out_features
        if isinstance(x, PendingNorm):
            if N % 128 == 0:
                r = ops.w8a8_gemv_norm(x.parts, x.residual, x.weight, x.eps, x.h, self.w_packed, self.w_scale,
                                       self.bias, N, K, glu_quant=True)
                if r is not None:
                    return QAct(*r)
            x = x.materialize()
        M = x.q.numel() // K
        quant = N % 128 == 0 and (glu_quant_rows(M) or M > 64)
        out = ops.w8a8_glu(x.q.reshape(-1, K), x.scale.reshape(-1), self.w_packed, self.w_scale, self.bias, N, K,
                           w_ref=self._wref(x.q), quant=quant)
        return QAct(*out) if quant else GroupQuantBF16(out)

    def geluq_rows_ok(self, M: int) -> bool:
        """Whether the fused up projection + GELU + grouped int8 quant takes M rows (GPU <= 64)."""
        return M <= 64 and self.out_features % 64 == 0 and not self.glu_blocked

    def pending_ln_ok(self, geluq: bool = False) -> bool:
        """Whether this projection's batch-1 GEMV can take a PendingLN (LayerNorm + int8 quant of bf16
        rows in its prologue; geluq: as the quantising GELU up projection)."""
        ok = self.w_packed.is_cuda and ops.gpu_path(self.w_packed) and not self.split_k_out \
            and not self.glu_blocked and self.in_features <= 4096 and self.in_features % 64 == 0
        return ok and self.out_features % (64 if geluq else 16) == 0

    def geluq(self, x: QAct, act: str) -> QAct:
        """GELU MLP front half in one launch (ops.w8a8_geluq): int8 h per (token, 64 columns).  A
        PendingLN input (batch 1) is normalised and quantised in the same kernel's prologue."""
        K, N = self.in_features, self.out_features
        if isinstance(x, PendingLN):
            r = ops.w8a8_gemv_ln(x.x, x.residual, x.weight, x.bias, x.eps, x.h, self.w_packed, self.w_scale,
                                 self.bias, N, K, geluq=act)
            if r is not None:
                return QAct(*r)
            x = x.materialize()
        q, s = ops.w8a8_geluq(x.q.reshape(-1, K), x.scale.reshape(-1), self.w_packed, self.w_scale, self.bias, N, K,
                              act, w_ref=self._wref(x.q))
        return QAct(q, s)

    def extra_repr(self):
        return f"{self.in_features}->{self.out_features}, bias={self.bias is not None}, W8A8 int8"


class LLMInt8Linear(nn.Module):
    takes_quantized_input = False
    graph_safe = False   # outlier-column discovery is data dependent (host sync on CPU), like bnb ...
    OUTLIER_CAP = 256    # ... on GPU ops/csrc/llmint8.hip finds the columns on the device: decode rows
    #                      (<= 16, one fused kernel, at most 256 columns) and any rows (uncapped)
    DECODE_ROWS = 16
    ONE_LAUNCH = True    # batch 1: ops/csrc/gemm_i8.hip l8_prologue (one launch per projection, K <= 12288)

    def pending_norm_ok(self, glu: bool = False):
        """Batch 1 on GPU: this projection takes the RMSNorm of a bf16 row x + residual in its one-launch
        GEMV's prologue ("x": a PendingLN with rms=True; Norm(defer="x"))."""
        return "x" if (self._device_ok() and self.ONE_LAUNCH and self.in_features <= 4096) else False

    def pending_ln_ok(self) -> bool:
        """Batch 1 on GPU: this projection takes the LayerNorm of x + residual in its prologue."""
        return self._device_ok() and self.ONE_LAUNCH and self.in_features <= 4096

    takes_pending_x = True           # MLP: hand a PendingLN to this projection instead of materialising

    def _device_ok(self) -> bool:
        K = self.in_features
        return ops.available() and self.w_packed.is_cuda and K % 32 == 0 and K <= 32768

    @property
    def graph_safe_rows(self) -> int:
        """Batch sizes up to which forward() runs without a host sync (graph-capturable): any on GPU."""
        return 1 << 30 if self._device_ok() else 0

    def __init__(self, in_features: int, out_features: int, bias: bool, threshold: float = 6.0, device=None,
                 dtype=torch.bfloat16):
        super().__init__()
        self.in_features, self.out_features, self.threshold = in_features, out_features, threshold
        kt, nt = (in_features + 63) // 64, (out_features + 15) // 16
        self.register_buffer("weight_i8", torch.zeros(out_features, in_features, dtype=torch.int8, device=device))
        self.register_buffer("w_packed", torch.zeros(nt * kt * 1024, dtype=torch.int8, device=device))
        self.register_buffer("SCB", torch.ones(out_features, dtype=torch.float32, device=device))
        self.register_buffer("bias", torch.zeros(out_features, dtype=dtype, device=device) if bias else None)
        self._weight_t = None          # int8 W^T for the device-side outlier path (built on first use)

    @classmethod
    @torch.no_grad()
    def from_float(cls, lin: Linear, threshold: float = 6.0) -> "LLMInt8Linear":
        w = lin.weight.float()
        scb = w.abs().amax(1).clamp_min(1e-8)              # bnb: per-row absmax (SCB)
        q = torch.round(w * (127.0 / scb[:, None])).clamp_(-127, 127).to(torch.int8)
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, threshold, device=w.device,
                dtype=lin.weight.dtype)
        m.load_int8(q, scb, lin.bias)
        return m

    @torch.no_grad()
    def _load_from_state_dict(self, *args, **kwargs):
        self._weight_t = None          # derived device copies follow the loaded weights
        super()._load_from_state_dict(*args, **kwargs)

    def load_int8(self, q, scb, bias=None):
        self._weight_t = None
        self.weight_i8.copy_(q)
        self.w_packed.copy_(ops.pack_int8_weight(q))
        self.SCB.copy_(scb.float())
        if bias is not None:
            self.bias.copy_(bias)

    def forward(self, x, add=None):
        out = self._forward(x)
        return out if add is None else out + add.view_as(out)

    def glu_norm(self, x: PendingLN):
        """Batch 1, [gate | up] rows: silu(gate) * up of the projection of RMSNorm(x + residual), one
        launch (bf16 [1, N / 2]); None when not taken (the caller materialises)."""
        return self._forward(x, glu=True) if (x.rms and self.out_features % 32 == 0) else None

    _ACT = {"gelu_tanh": 1, "gelu": 2}

    def gelu_fused(self, x, act: str):
        """Batch 1: gelu (tanh / erf) of this projection in the same launch (bf16 [1, N]), over a bf16
        row or a PendingLN; None when not taken."""
        if act not in self._ACT:
            return None
        if isinstance(x, PendingLN):
            return self._forward(x, act=self._ACT[act])
        if isinstance(x, torch.Tensor) and x.dim() == 2 and x.shape[0] == 1 and x.dtype == torch.bfloat16 \
                and x.is_cuda and ops.gpu_path(x) and self._device_ok() and self.ONE_LAUNCH \
                and self.in_features <= 4096:
            return self._forward(x, act=self._ACT[act])
        return None

    def _forward(self, x, glu: bool = False, act: int = 0):
        if isinstance(x, PendingLN):
            y = None
            K, N = self.in_features, self.out_features
            if (x.x.shape[0] == 1 and x.x.is_cuda and ops.gpu_path(x.x) and x.x.dtype == torch.bfloat16
                    and self._device_ok() and self.ONE_LAUNCH and K <= 4096):
                C = ops.ext()
                if self._weight_t is None or self._weight_t.device != x.x.device:
                    self._weight_t = self.weight_i8.t().contiguous()
                    self._w_deq = self.SCB / 127.0
                y = C.llmint8_gemv_norm(x.x.contiguous(), x.residual.contiguous() if x.residual is not None else None,
                                        x.weight, x.bias, x.eps, not x.rms, x.h, x.y, self.threshold, self.w_packed,
                                        self._w_deq, self.bias, self._weight_t, self.SCB, N, glu, act)
            if y is not None or glu or act:
                return y
            x = x.materialize()
        if isinstance(x, QAct):
            x = (x.q.float() * x.scale[..., None]).to(torch.bfloat16)
        K, N = self.in_features, self.out_features
        shp = x.shape[:-1]
        x2 = x.reshape(-1, K)
        if x2.is_cuda and ops.gpu_path(x2) and x2.dtype == torch.bfloat16 and self._device_ok():
            # outlier columns found on the device (llmint8.hip), no host sync at any row count
            C = ops.ext()
            if self._weight_t is None or self._weight_t.device != x2.device:
                self._weight_t = self.weight_i8.t().contiguous()          # W^T: outlier columns as rows
                self._w_deq = self.SCB / 127.0
            x2 = x2.contiguous()
            if x2.shape[0] == 1 and K <= 12288 and K % 64 == 0 and self.ONE_LAUNCH:
                # batch 1: outlier discovery, quantisation and the outlier part inside the GEMV
                out = C.llmint8_gemv(x2, self.threshold, self.w_packed, self._w_deq, self.bias, self._weight_t,
                                     self.SCB, N, act)
                if out is not None:
                    return out.view(*shp, N)
                if act:
                    return None
            if x2.shape[0] <= self.DECODE_ROWS:
                q, sa, cols, xo, count = C.llmint8_prep(x2, self.threshold, self.OUTLIER_CAP)
                out = ops.w8a8_linear(q, sa, self.w_packed, self._w_deq, self.bias, N, K)
                C.llmint8_outlier(out, xo, cols, count, self._weight_t, self.SCB)
            else:
                q, sa, cols, count = C.llmint8_prep_rows(x2, self.threshold)
                out = ops.w8a8_linear(q, sa, self.w_packed, self._w_deq, self.bias, N, K)
                C.llmint8_outlier_rows(out, x2, cols, count, self._weight_t, self.SCB)
            return out.view(*shp, N)
        cols = (x2.abs() > self.threshold).any(0).nonzero().flatten()
        w_scale = self.SCB / 127.0
        if cols.numel() > 0:
            x_in = x2.clone()
            x_in[:, cols] = 0
            w_out = (self.weight_i8[:, cols].float() * w_scale[:, None]).to(x.dtype)
            out_o = x2[:, cols] @ w_out.t()
        else:
            x_in, out_o = x2, None
        q, s = ops.quant_per_token(x_in.contiguous())
        out = ops.w8a8_linear(q, s, self.w_packed, w_scale, self.bias, N, K,
                              w_ref=None if q.is_cuda else self.weight_i8, out_dtype=x.dtype)
        if out_o is not None:
            out = (out.float() + out_o.float()).to(out.dtype)
        return out.view(*shp, N)

    def extra_repr(self):
        return f"{self.in_features}->{self.out_features}, LLM.int8 threshold={self.threshold}"


class CPUDynamicLinear(nn.Module):
    """torch dynamic-quantised qint8 linear on CPU (reference try.py:205 equivalent)."""
    takes_quantized_input = False
    graph_safe = False

    def __init__(self, lin: Linear):
        super().__init__()
        self.in_features, self.out_features = lin.in_features, lin.out_features
        f = nn.Linear(lin.in_features, lin.out_features, bias=lin.bias is not None)
        with torch.no_grad():
            f.weight.copy_(lin.weight.float().cpu())
            if lin.bias is not None:
                f.bias.copy_(lin.bias.float().cpu())
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            self.q = torch.ao.quantization.quantize_dynamic(nn.Sequential(f), {nn.Linear}, dtype=torch.qint8)[0]
        self.out_dtype = lin.weight.dtype

    def forward(self, x, add=None):
        if isinstance(x, QAct):
            x = x.q.float() * x.scale[..., None]
        out = self.q(x.float()).to(self.out_dtype)
        return out if add is None else out + add.view_as(out).to(out.dtype)


def enable_fused_glu(model) -> int:
    """Block the W8A8 gate_up projections of SwiGLU layers (F % 64 == 0) so the decode MLP runs
    as GEMV+SwiGLU -> down GEMV with in-kernel per-group quant (two launches instead of three).
    Returns the number of layers changed."""
    cfg = model.cfg
    n = 0
    if cfg.is_glu and cfg.act == "silu_glu" and cfg.intermediate_size % 64 == 0:
        for layer in model.layers:
            if layer.mlp is None:
                continue
            up = layer.mlp.up
            if isinstance(up, W8A8Linear) and isinstance(layer.mlp.down, W8A8Linear) and not up.glu_blocked:
                up.block_glu_()
                n += 1
    enable_split_k_outputs(model)
    return n


# EDGELLM_SPLITK: 0 turns the split-K decode outputs off, 1 = automatic split count, N > 1 forces N
SPLIT_K = int(os.environ.get("EDGELLM_SPLITK", "1"))


def enable_split_k_outputs(model) -> int:
    """Sequential-residual RMSNorm decoders (Llama): the o and down projections feed an RMSNorm
    (or the stage exit), so on GPU their decode GEMVs emit split-K partial slices that the norm
    kernel sums — each workgroup then reads 1/S of the activation matrix instead of all of it."""
    cfg = model.cfg
    if not SPLIT_K or cfg.parallel_residual or cfg.norm != "rms":
        return 0
    n = 0
    for layer in model.layers:
        for lin in [m for m in (layer.attn and layer.attn.o, layer.mlp and layer.mlp.down) if m is not None]:
            if isinstance(lin, W8A8Linear) and lin.in_features % 64 == 0:
                lin.split_k_out = SPLIT_K
                n += 1
    return n

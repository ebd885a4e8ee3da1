"""edgellm op layer: every hot op of the decoder, one function each.

GPU tensors run the hand-written CDNA4 kernels in ``ops/csrc`` (compiled in-tree to
``ops/_C*.so`` by ``ops/build.py``); CPU tensors run the fp32 PyTorch reference in
``ops/_ref.py`` (CPU plumbing configs and unit tests).  There is no silent fallback on the
GPU: if the extension is missing or was built for another arch, GPU calls raise.
Setting ``EDGELLM_REF_ON_GPU=1`` explicitly routes GPU tensors through the reference (used
only for A/B numerics checks).
"""
from __future__ import annotations

import importlib
import os
from typing import Optional, Tuple

import torch

from . import _ref

_C = None
_C_ERR: Optional[BaseException] = None


def _load():
    global _C, _C_ERR
    if _C is None and _C_ERR is None:
        try:
            _C = importlib.import_module(__name__ + "._C")
        except BaseException as e:  # noqa: BLE001 - re-raised on first GPU use
            _C_ERR = e
        else:
            apply_tune(os.environ.get("EDGELLM_TUNE", ""))
    return _C


def apply_tune(spec: str) -> None:
    """Kernel tuning knobs from ``name=a[,b];name=a`` (``EDGELLM_TUNE``): A/B a launcher choice
    at model level without a rebuild (names: the extension's ``tune`` table)."""
    for item in filter(None, (t.strip() for t in spec.replace(";", " ").split())):
        name, _, vals = item.partition("=")
        v = [int(x) for x in vals.split(",") if x] + [0, 0]
        _C.tune(name, v[0], v[1])


def ext():
    """The compiled extension; raises with the import error when it is unavailable."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "edgellm HIP extension not available (build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            f" or ops/build.py): {_C_ERR!r}")
    return m


def available() -> bool:
    return _load() is not None


_REF_ON_GPU = os.environ.get("EDGELLM_REF_ON_GPU", "0") == "1"


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda and not _REF_ON_GPU


# --------------------------------------------------------------------------- norms


def gpu_path(t: torch.Tensor) -> bool:
    """True when ``t`` runs through the HIP kernels (not the reference ops)."""
    return _gpu(t)


def rms_norm_parts(parts, residual, weight, eps, quant: bool, packed: bool = False):
    """RMSNorm of the in-order sum of split-K partial slices parts [S, M, H] (fp32) rounded to bf16
    (+ residual): returns (y bf16 | q int8, per-token scale | None, h = bf16 sum (+ residual)).
    ``packed`` (quant, 129-256 rows): q is the [M, H] view of a fragment-packed [256, H] buffer for
    the 256-row decode GEMM (``w8a8_r256``)."""
    return ext().rms_norm_parts(parts, residual, weight, eps, 2 if (quant and packed) else int(quant))


def r256_ok(M: int, N: int, K: int) -> bool:
    """Whether the packed-activation 256-row decode GEMM (gemm_i8.hip w8a8_r256_kernel) takes this
    W8A8 shape on the GPU (129-256 rows; tune knob ``r256_packed``)."""
    return 128 < M <= 256 and available() and bool(ext().r256_ok(M, N, K))


def w8a8_r256(qx_packed, x_scale, w_packed, w_scale, bias, N: int, K: int):
    """W8A8 GEMM of a fragment-packed activation (``rms_norm_quant(..., packed=True)``) at 129-256
    rows -> bf16 [M, N]; None when the packed kernel does not take the shape."""
    out = ext().w8a8_r256(qx_packed, x_scale.reshape(-1), w_packed, w_scale, bias, N, K)
    return out if out.numel() else None


def unpack_a(q_packed, M: int, K: int):
    """Row-major int8 [M, K] of a fragment-packed activation (piece (rb, kt) = 16 rows x 64 k at
    (rb * K/64 + kt) * 1024, lane l's 16 B = row 16 rb + (l & 15), k 64 kt + 16 (l >> 4) ..)."""
    KT = K // 64
    buf = torch.as_strided(q_packed, (256 * K,), (1,))
    t = buf.view(16, KT, 4, 16, 16)                     # [rb, kt, k16 group, row in rb, byte]
    return t.permute(0, 3, 1, 2, 4).reshape(256, K)[:M].contiguous()


# rows up to which decode norms move into the next GEMV's prologue (kernel: <= 4).  Round 4 (the
# prologue's loads queued behind the weights): batch 1 2.10 -> 1.96 ms, 4 rows 2.167 -> 2.179 ms
# (slower), so 1.  Round 6 (prologue loads first, profiles/norm_fuse_rows_ab_r6.jsonl): Llama-2-7B
# W8A8 2 rows 2.108 -> 1.919 ms, 4 rows 2.155 -> 2.097; Llama-3.2-1B bf16 4 rows 0.811 -> 0.758: 4.
NORM_FUSE_MAX_ROWS = int(os.environ.get("EDGELLM_NORM_FUSE_ROWS", "4"))


def gemv_norm_ok(parts) -> bool:
    """Whether a decode W8A8 GEMV can take the RMSNorm of these split-K slices [S, M, K] in its
    prologue (gemm_i8.hip NormIn: M <= 4, K 2048 / 4096, S <= 4; tune knob ``gemv_norm``)."""
    return parts.is_cuda and parts.dim() == 3 and 1 <= parts.shape[1] <= min(4, NORM_FUSE_MAX_ROWS) \
        and 1 <= parts.shape[0] <= 4 \
        and parts.shape[2] in (2048, 4096) and available() and bool(ext().gemv_norm_on())


def gemv_bf16_norm(parts, residual, gamma, eps: float, res_out, packed, bias, N: int, glu: bool = False):
    """16-bit decode GEMV (M <= 4 rows) over RMSNorm(sum(parts) + residual (None: no residual)),
    the norm in the GEMV's prologue (gemv_bf16.hip norm16_prologue, bit-identical to the norm
    kernel); the new residual rows go to ``res_out``.  ``packed``: ``pack_bf16_weight(W)``;
    ``glu``: W = [gate | up], returns silu(gate) * up [M, N / 2].  None when no kernel takes it."""
    return ext().gemv_bf16_norm(parts, residual.contiguous() if residual is not None else None, gamma, eps, res_out,
                                packed, bias, N, 1 if glu else 0)


def gemv_ln_ok(x) -> bool:
    """Whether a decode 16-bit GEMV can take the LayerNorm of these rows x [M, K] (+ residual) in
    its prologue (gemv_bf16.hip ln16_prologue: M <= NORM_FUSE_MAX_ROWS, K <= 4096, K % 64 == 0)."""
    return x.is_cuda and x.dim() == 2 and 1 <= x.shape[0] <= min(4, NORM_FUSE_MAX_ROWS) and x.shape[1] <= 4096 \
        and x.shape[1] % 64 == 0 and x.dtype in (torch.bfloat16, torch.float16) and x.is_contiguous() \
        and available() and bool(ext().gemv_norm_on())


_LN_EPI = {None: 0, "gelu_tanh": 2, "gelu": 3}


def gemv_bf16_ln(x, residual, gamma, beta, eps: float, res_out, packed, bias, N: int, act: Optional[str] = None,
                 y_out=None):
    """16-bit decode GEMV (M <= 4 rows) over LayerNorm(x + residual (None: none)) with the norm in
    its prologue (bit-identical to the norm kernel); x + residual goes to ``res_out``, the
    normalised rows to ``y_out`` when given (a second consumer's input); ``act``: None /
    "gelu_tanh" / "gelu" epilogue.  None when no kernel takes the shape."""
    return ext().gemv_bf16_ln(x, residual.contiguous() if residual is not None else None, gamma, beta, eps, res_out,
                              packed, bias, N, _LN_EPI[act], y_out)


def w8a8_gemv_ln(x, residual, gamma, beta, eps: float, res_out, w_packed, w_scale, bias, N: int, K: int,
                 geluq: Optional[str] = None):
    """W8A8 decode GEMV (M <= 4 rows) over LayerNorm(x + residual) of bf16 rows, int8 per token, the
    norm in its prologue (bit-identical to layer_norm_quant); x + residual goes to ``res_out``.
    Returns bf16 y [M, N], or with ``geluq`` ("gelu_tanh" / "gelu") the quantising GELU's
    (q [M, N], scales [N/64, 16]).  None when no kernel takes the shape."""
    epi = 0 if geluq is None else (4 if geluq == "gelu_tanh" else 5)
    r = ext().w8a8_gemv_ln(x, residual.contiguous() if residual is not None else None, gamma, beta, eps, res_out,
                           w_packed, w_scale, bias, N, K, epi)
    if r is None:
        return None
    return r if geluq is not None else r[0]


def w8a8_gemv_norm(parts, residual, gamma, eps: float, res_out, w_packed, w_scale, bias, N: int, K: int,
                   glu_quant: bool = False):
    """Decode W8A8 GEMV (M <= 4 rows) over RMSNorm(sum(parts) + residual (None: no residual)), per-token int8, with
    the norm in the GEMV's prologue; the new residual rows go to ``res_out``.  Returns bf16 y [M, N],
    or with ``glu_quant`` (16-blocked gate_up) the quantising SwiGLU's (q [M, N/2], scales
    [N/128, 16]);
    None when no kernel takes the shape (the caller runs the norm kernel instead)."""
    r = ext().w8a8_gemv_norm(parts, residual.contiguous() if residual is not None else None, gamma, eps, res_out,
                             w_packed, w_scale, bias, N, K, 2 if glu_quant else 0)
    if r is None:
        return None
    return r if glu_quant else r[0]


def decode_rows_ok(M: int, K: int, splits: int = 1) -> bool:
    """Whether the decode GEMV family (grouped scales, split-K, quantising GLU) takes M rows at
    this K: every K up to 64 rows; 65-128 rows (two micro-batches in one: the ring2 kernel) for
    K % 128 == 0 (split-K: >= 4 stages of 128 k per slice); 129-256 rows (one 256-row
    micro-batch: the row-split ring2 kernels, split-K count fixed per K) for K % 128 == 0."""
    if M <= 64:
        return True
    if M > 256 or not available():
        return False
    if M > 128:
        return bool(ext().rows256_ok(K))
    return bool(ext().rows128_ok(K, splits))


# Activation scales of the o / down inputs at 129-256 decode rows: "group" = per (token, 64) from
# the fused producers (attention epilogue, quantising SwiGLU GEMM), folded per k-tile in the GEMM;
# "token" = bf16 producer output + a per-token quant launch, no fold in the GEMM (A/B knob)
DEC256_GROUP = os.environ.get("EDGELLM_DEC256_SCALES", "group") == "group"


def group_scale_rows_ok(M: int) -> bool:
    """Whether decode producers emit per-(token, 64) scales at M rows (always up to 128)."""
    return M <= 128 or DEC256_GROUP


def w8a8_linear_splitk(qx, x_scale, w_packed, w_scale, bias, N: int, K: int, splits: int = 0):
    """Split-K W8A8 GEMV (GPU, K % 64 == 0, M <= 64 or ``decode_rows_ok(M, K, 4)``): fp32 partial
    slices [S, M, N]."""
    return ext().w8a8_gemm_splitk(qx, x_scale, w_packed, w_scale, bias, N, K, splits)


def rms_norm(x, weight, eps, residual=None):
    if _gpu(x):
        y, _, r = ext().norm(x, residual, weight, None, eps, True, False)
        return y, r
    return _ref.rms_norm(x, weight, eps, residual)


def layer_norm(x, weight, bias, eps, residual=None):
    if _gpu(x):
        y, _, r = ext().norm(x, residual, weight, bias, eps, False, False)
        return y, r
    return _ref.layer_norm(x, weight, bias, eps, residual)


def rms_norm_quant(x, weight, eps, residual=None, packed: bool = False):
    """``packed`` (GPU, 129-256 rows): the int8 rows fragment-packed for ``w8a8_r256``."""
    if _gpu(x):
        return ext().norm(x, residual, weight, None, eps, True, 2 if packed else 1)
    return _ref.rms_norm_quant(x, weight, eps, residual)


def layer_norm_quant(x, weight, bias, eps, residual=None):
    if _gpu(x):
        return ext().norm(x, residual, weight, bias, eps, False, 1)
    return _ref.layer_norm_quant(x, weight, bias, eps, residual)


def w8a8_prefill_glu(qx, x_scale, w_packed, w_scale, bias, N: int, K: int):
    """Prefill gate_up of a 16-blocked SwiGLU layer with silu(g) * u in the GEMM epilogue (GPU x32
    kernel): bf16 h [M, N / 2], or None when the kernel does not take the shape."""
    if not gpu_path(qx):
        return None
    return ext().w8a8_prefill_glu(qx, x_scale, w_packed, w_scale, bias, N, K)


def quant_per_token(x):
    if _gpu(x):
        return ext().quant(x)
    return _ref.quant_per_token(x)


# --------------------------------------------------------------------------- activations
_ACT_MODE = {"silu_glu": 0, "gelu_tanh": 1, "gelu": 2, "silu_glu_blocked": 3}


def activation(x, act: str):
    """``silu_glu``: x = [gate | up]; ``silu_glu_blocked``: 16-blocked [gate(16) | up(16)] rows
    (the packing of W8A8 gate_up weights, see quant.linear.W8A8Linear.glu_blocked)."""
    if _gpu(x):
        return ext().act(x, _ACT_MODE[act], False)[0]
    if act == "silu_glu":
        return _ref.silu_mul(x)
    if act == "silu_glu_blocked":
        return _ref.silu_mul(_ref.unblock_glu(x))
    return _ref.gelu(x, "tanh" if act == "gelu_tanh" else "none")


def activation_quant(x, act: str):
    if _gpu(x):
        return ext().act(x, _ACT_MODE[act], True)
    if act == "silu_glu":
        return _ref.silu_mul_quant(x)
    if act == "silu_glu_blocked":
        return _ref.silu_mul_quant(_ref.unblock_glu(x))
    return _ref.gelu_quant(x, "tanh" if act == "gelu_tanh" else "none")


# --------------------------------------------------------------------------- rope / attention


def rope_kv_write(qkv, start_pos, rope, k_cache, v_cache, num_heads, num_kv_heads, head_dim, rotary_dim,
                  k2=None, v2=None, split: int = -1, cpos2=None):
    """RoPE on q/k + KV append.  With ``split`` (HeadInfer), kv heads >= split go to (k2, v2)
    at positions cpos2[b] + t instead of the main cache."""
    if _gpu(qkv):
        return ext().rope_kv_write(qkv, start_pos, rope, k_cache, v_cache, num_heads, num_kv_heads, head_dim,
                                   rotary_dim, k2, v2, split, cpos2)
    return _ref.rope_kv_write(qkv, start_pos, rope, k_cache, v_cache, num_heads, num_kv_heads, head_dim, rotary_dim,
                              k2, v2, split, cpos2)


COPY_TRANSPORTS = {0: "none", 1: "kernel", 2: "dma", 3: "torch"}


def copy_head_block(dst, src, mode: int = 0) -> str:
    """Async strided copy of a [B, c, L, D] KV head block (pinned host <-> device) on the
    current stream.  ``mode`` 0 = auto (rows >= 64 KiB on the copy engines, shorter rows by the
    copy kernel over mapped pinned memory), 1 = kernel, 2 = copy engines.  Returns the transport
    used ("kernel" | "dma" | "torch" on CPU)."""
    if (dst.is_cuda or src.is_cuda) and not _REF_ON_GPU:
        return COPY_TRANSPORTS[int(ext().copy_head_block(dst, src, int(mode)))]
    dst.copy_(src)
    return "torch"


def decode_attention(q, k_cache, v_cache, seq_lens, scale, max_len_hint: Optional[int] = None):
    if _gpu(q):
        hint = int(max_len_hint) if max_len_hint is not None else int(k_cache.shape[2])
        return ext().decode_attn(q, k_cache, v_cache, seq_lens, scale, hint)
    return _ref.decode_attention(q, k_cache, v_cache, seq_lens, scale)


def decode_attention_fused(qkv, start_pos, rope, k_cache, v_cache, seq_lens, num_heads: int, scale: float,
                           max_len_hint: int, rotary_dim: int, quant_out: bool = False):
    """Decode step straight from the QKV projection: RoPE on q, append of the new k/v at
    ``start_pos`` and attention over ``[0, seq_lens)`` in one launch.  ``quant_out`` returns
    ``(int8 [B, Hq*D], scales [Hq*D/64, Mpad])`` for a W8A8 o-projection, else ``(bf16 [B, Hq, D], None)``."""
    Hkv, D = k_cache.shape[1], k_cache.shape[3]
    if _gpu(qkv):
        return ext().decode_attn_fused(qkv, start_pos, rope if rotary_dim else None, k_cache, v_cache, seq_lens,
                                       num_heads, scale, int(max_len_hint), rotary_dim, quant_out)
    q = _ref.rope_kv_write(qkv, start_pos, rope if rotary_dim else None, k_cache, v_cache, num_heads, Hkv, D,
                           rotary_dim)
    out = _ref.decode_attention(q.view(qkv.shape[0], num_heads, D), k_cache, v_cache, seq_lens, scale)
    if quant_out:
        return _ref.quant_per_group(out.reshape(qkv.shape[0], num_heads * D))
    return out, None


def decode_attention_fused_i8(qkv, start_pos, rope, k_cache, v_cache, k_scale, v_scale, seq_lens, num_heads: int,
                              scale: float, max_len_hint: int, rotary_dim: int, quant_out: bool = False):
    """``decode_attention_fused`` over an int8 KV cache (int8 [B, Hkv, S, D] + fp32 scales
    [B, Hkv, S]): the new token is quantised per (token, head) in the same launch
    (ops/csrc/attn_decode_i8.hip)."""
    Hkv, D = k_cache.shape[1], k_cache.shape[3]
    if _gpu(qkv):
        return ext().decode_attn_i8(qkv, start_pos, rope if rotary_dim else None, k_cache, v_cache, k_scale, v_scale,
                                    seq_lens, num_heads, scale, int(max_len_hint), rotary_dim, quant_out)
    q = _ref.rope_kv_write_i8(qkv, start_pos, rope if rotary_dim else None, k_cache, v_cache, k_scale, v_scale,
                              num_heads, Hkv, D, rotary_dim)
    S = int(seq_lens.max().item())
    kf = _ref.dequant_kv(k_cache[:, :, :S], k_scale[:, :, :S])
    vf = _ref.dequant_kv(v_cache[:, :, :S], v_scale[:, :, :S])
    out = _ref.decode_attention(q.view(qkv.shape[0], num_heads, D).float(), kf, vf, seq_lens, scale).to(qkv.dtype)
    if quant_out:
        return _ref.quant_per_group(out.reshape(qkv.shape[0], num_heads * D))
    return out, None


def kv_quant_append(src, start_pos, T: int, cache, scales):
    """Quantise bf16 rows ``src[b, h, start_pos[b] + t]`` (t < T) into an int8 cache + scales."""
    if _gpu(src):
        return ext().kv_quant_append(src, start_pos, int(T), cache, scales)
    for b in range(src.shape[0]):
        p0 = int(start_pos[b])
        q, s = _ref.quant_kv_rows(src[b, :, p0:p0 + T])
        cache[b, :, p0:p0 + T] = q
        scales[b, :, p0:p0 + T] = s


def kv_dequant(cache, scales, dst, T: int):
    """``dst[:, :, :T] = cache[:, :, :T] * scales[:, :, :T, None]`` (int8 KV rows -> bf16 scratch),
    one kernel on GPU (no fp32 temporaries)."""
    if T <= 0:
        return
    if _gpu(cache):
        return ext().kv_dequant(cache, scales, dst, int(T))
    dst[:, :, :T] = _ref.dequant_kv(cache[:, :, :T], scales[:, :, :T]).to(dst.dtype)


def prefill_attention(q, k_cache, v_cache, start_pos, scale, causal=True):
    if _gpu(q):
        return ext().prefill_attn(q, k_cache, v_cache, start_pos, scale, causal)
    return _ref.prefill_attention(q, k_cache, v_cache, start_pos, scale, causal)


# --------------------------------------------------------------------------- INT8 GEMM


def pack_int8_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] int8 -> MFMA-fragment-packed 1 KiB tiles (see csrc/gemm_i8.hip header).
    N is padded to 16 and K to 64 with zeros."""
    N, K = w.shape
    NT, KT = (N + 15) // 16, (K + 63) // 64
    wp = torch.zeros(NT * 16, KT * 64, dtype=torch.int8, device=w.device)
    wp[:N, :K] = w
    # [NT, n16, KT, kc4, b16] -> [NT, KT, kc4, n16, b16]
    return wp.view(NT, 16, KT, 4, 16).permute(0, 2, 3, 1, 4).contiguous().view(-1)


def unpack_int8_weight(wp: torch.Tensor, N: int, K: int) -> torch.Tensor:
    NT, KT = (N + 15) // 16, (K + 63) // 64
    w = wp.view(NT, KT, 4, 16, 16).permute(0, 3, 1, 2, 4).reshape(NT * 16, KT * 64)
    return w[:N, :K].contiguous()


# rows the bf16 decode GEMV takes (gemv_bf16.hip handles up to 64: 4 row blocks per weight read)
BF16_GEMV_MAX_ROWS = int(os.environ.get("EDGELLM_BF16_GEMV_ROWS", "16"))


# rows the bf16 ring GEMM (gemm_i8.hip ring2 kernel, bf16 MFMA) takes above the GEMV
BF16_RING_MAX_ROWS = 256


def bf16_decode_mode(x: torch.Tensor, weight: torch.Tensor, glu: bool = False, split: bool = False) -> int:
    """Which HIP decode kernel ``linear_bf16`` runs for this call (bf16, or fp16 for the GEMV): 1 = ``gemv_bf16.hip`` (<=
    ``BF16_GEMV_MAX_ROWS`` rows), 2 = the bf16 ring GEMM (up to 256 rows, from the extension's
    ``bf16_ring_min_rows`` (65), or from 17 rows for the fused SwiGLU, split-K outputs and
    LM-head-wide N >= 16384), 0 = none (hipBLASLt; measured ahead of the ring on qkv at 17-64
    rows).  GPU, bf16, K % 64 == 0, N % 16 == 0 (% 32 for
    the fused GLU)."""
    K = x.shape[-1]
    if not (_gpu(x) and x.dtype in (torch.bfloat16, torch.float16) and weight.dtype == x.dtype
            and x.is_contiguous() and K % 64 == 0 and weight.shape[0] % (32 if glu else 16) == 0):
        return 0
    M = x.numel() // max(K, 1)
    if 0 < M <= BF16_GEMV_MAX_ROWS:
        return 1
    if x.dtype != torch.bfloat16:          # fp16: the GEMV only (the ring GEMM is bf16)
        return 0
    lo = ext().bf16_ring_min_rows()
    if glu or split or weight.shape[0] >= 16384:
        # SwiGLU, split-K (o / down) and LM-head-wide N: the ring is ahead from 17 rows
        # (profiles/bench_ops_r3_bf16ring_b.json); narrow plain outputs (qkv) from the default
        lo = min(lo, BF16_GEMV_MAX_ROWS + 1)
    if lo <= M <= BF16_RING_MAX_ROWS:
        return 2
    return 0


def bf16_gemv_ok(x: torch.Tensor, weight: torch.Tensor, glu: bool = False) -> bool:
    """Whether ``linear_bf16`` runs a HIP decode kernel for this call (``bf16_decode_mode``)."""
    return bf16_decode_mode(x, weight, glu) != 0


def pack_bf16_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] bf16 (or fp16) -> MFMA-fragment order for ``gemv_bf16.hip``: 1 KiB tiles of 16 rows x 32 k,
    lane l holding W[16 nt + (l & 15)][32 kt + 8 (l >> 4) .. +8] (N % 16 == 0, K % 32 == 0)."""
    N, K = w.shape
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().view(-1)


_GEMV_EPI = {None: 0, "silu_glu": 1, "gelu_tanh": 2, "gelu": 3}


def linear_bf16(x, weight, bias=None, glu: bool = False, act: Optional[str] = None,
                packed: Optional[torch.Tensor] = None, add: Optional[torch.Tensor] = None):
    """16-bit projection (bf16, or fp16 for the fp16 agents: the GEMV's fp16 MFMA instantiation).  Decode-sized inputs on GPU take ``gemv_bf16.hip`` on the fragment-packed
    weight (``packed``: the layer's cached ``pack_bf16_weight(weight)``; packed per call when
    absent); ``glu``: weight = [gate | up] and the result is silu(gate) * up; ``act``
    "gelu_tanh" / "gelu": the activation of the bf16 output in the same kernel.  Everything else
    is ``F.linear`` (hipBLASLt on GPU) followed by the activation op.  ``add`` (bf16, the output's
    shape; plain outputs only): returns bf16(y + add), in the GEMV epilogue where it runs."""
    if glu:
        act = "silu_glu"
    assert add is None or act is None, "addend: plain outputs only"
    mode = bf16_decode_mode(x, weight, glu)
    if mode == 1 or (mode == 2 and act in (None, "silu_glu")):
        wp = packed if packed is not None else pack_bf16_weight(weight)
        if mode == 1:
            return ext().gemv_bf16(x, wp, bias, weight.shape[0], _GEMV_EPI[act], add)
        y = ext().gemm_bf16_ring(x, wp, bias, weight.shape[0], 1 if glu else 0, 0)
        return y if add is None else y + add
    if mode == 2:           # GELU MLPs: ring GEMM, then the activation kernel
        wp = packed if packed is not None else pack_bf16_weight(weight)
        return activation(ext().gemm_bf16_ring(x, wp, bias, weight.shape[0], 0, 0), act)
    y = torch.nn.functional.linear(x, weight, bias)
    y = y if act is None else activation(y, act)
    return y if add is None else y + add


def w8a8_linear(qx, x_scale, w_packed, w_scale, bias, N: int, K: int, w_ref: Optional[torch.Tensor] = None,
                out_dtype=torch.bfloat16, add: Optional[torch.Tensor] = None):
    """INT8 x INT8 -> int32 MFMA GEMM with per-channel weight dequant (+bias) -> bf16.
    ``x_scale`` is per token ([M]) or per (token, 64-column group) ([K/64, Mpad], M <= 64, from the
    fused producers).  ``out_dtype`` applies on CPU, where fp16/fp32 agents run; ``w_ref``
    (canonical [N, K]) is only needed by the CPU path.  ``add``: returns y + add (the other branch
    of a parallel-residual block), in the GEMV epilogue at decode rows on GPU."""
    if _gpu(qx):
        return ext().w8a8_gemm(qx, x_scale, w_packed, w_scale, bias, N, K,
                               None if add is None else add.contiguous())
    w = w_ref if w_ref is not None else unpack_int8_weight(w_packed, N, K)
    shp = qx.shape[:-1]
    xs = x_scale if x_scale.dim() == 2 else x_scale.reshape(-1)
    out = _ref.w8a8_linear(qx.reshape(-1, K), xs, w, w_scale, bias, out_dtype).view(*shp, N)
    return out if add is None else out + add.view(*shp, N).to(out.dtype)


def w8a8_glu(qx, x_scale, w_packed, w_scale, bias, N: int, K: int, w_ref: Optional[torch.Tensor] = None,
             quant: bool = False):
    """Fused decode MLP front half: gate_up projection (16-blocked rows, N = 2F) -> silu(g) * u
    (one launch on GPU, M <= 64; gate/up rounded to bf16 as the GEMM output).

    Returns bf16 h [M, F], or with ``quant`` (N % 128 == 0) the int8 per-(token, 64 features)
    quantisation of h computed in the same kernel: (q [M, F], scales [F/64, Mpad])."""
    if _gpu(qx):
        if quant:
            return ext().w8a8_gemm_gluq(qx, x_scale, w_packed, w_scale, bias, N, K)
        return ext().w8a8_gemm_glu(qx, x_scale, w_packed, w_scale, bias, N, K)
    w = w_ref if w_ref is not None else unpack_int8_weight(w_packed, N, K)
    y = _ref.w8a8_linear(qx.reshape(-1, K), x_scale.reshape(-1), w, w_scale, bias, torch.bfloat16)
    if quant:
        g, u = _ref.unblock_glu(y).float().chunk(2, dim=-1)
        return _ref.quant_per_group(torch.nn.functional.silu(g) * u)
    return _ref.silu_mul(_ref.unblock_glu(y))


def w8a8_geluq(qx, x_scale, w_packed, w_scale, bias, N: int, K: int, act: str = "gelu_tanh",
               w_ref: Optional[torch.Tensor] = None):
    """Fused decode GELU MLP front half (M <= 64, N % 64 == 0): up projection -> gelu (tanh / erf)
    of its bf16 output -> int8 per (token, 64 columns), one launch on GPU: (q [M, N], scales
    [N/64, Mpad]) for the down projection's grouped-scale GEMV."""
    if _gpu(qx):
        return ext().w8a8_gemm_geluq(qx, x_scale, w_packed, w_scale, bias, N, K, act == "gelu_tanh")
    w = w_ref if w_ref is not None else unpack_int8_weight(w_packed, N, K)
    y = _ref.w8a8_linear(qx.reshape(-1, K), x_scale.reshape(-1), w, w_scale, bias, torch.bfloat16)
    return _ref.quant_per_group(_ref.gelu(y, "tanh" if act == "gelu_tanh" else "none"))


def quant_per_group(x):
    """Per-(token, 64 columns) int8: (q [M, K], scales [K/64, Mpad]) — the decode-GEMV input
    layout (ops/csrc/rowwise.hip::group_quant_kernel on GPU)."""
    if _gpu(x):
        return ext().group_quant(x)
    return _ref.quant_per_group(x)


# --------------------------------------------------------------------------- sampling / misc


def _logits32(logits):
    """The sampler reads bf16 or fp32 logits; fp16 logits (fp16 agents) are widened to fp32 first,
    as HF's generate does before its logits processors."""
    return logits.float() if logits.dtype == torch.float16 else logits


def sample(logits, seen, temperature, top_k, top_p, repetition_penalty, rng: torch.Tensor,
           do_sample: bool = True):
    """Fused sampler. ``rng`` = int32 tensor [seed, step] on the logits' device (the step is
    read on device so the launch is graph-capturable)."""
    if _gpu(logits):
        logits = _logits32(logits)
        out = ext().sample(logits, seen, float(temperature), int(top_k or 0), float(top_p if top_p is not None else 1.0),
                           float(repetition_penalty), bool(do_sample), rng)
        if out.numel() > 0 or logits.shape[0] == 0:
            return out
        # top-p without top-k (or top-k > 1024): needs a full sort -> torch path on device
        seed, step = (int(v) for v in rng.tolist())
        tok = _ref.sample(logits, seen, temperature, top_k, top_p, repetition_penalty, seed, step, do_sample)
        if seen is not None:
            seen.scatter_(1, tok[:, None], 1)
        return tok
    seed, step = (int(v) for v in rng.tolist())
    tok = _ref.sample(logits, seen, temperature, top_k, top_p, repetition_penalty, seed, step, do_sample)
    if seen is not None:
        seen.scatter_(1, tok[:, None], 1)
    return tok


# --------------------------------------------------------------------------- vocab-sharded sampling
SHARD_CCAP = 128          # candidates per chunk list (sampler.hip CCAP): top-k shards up to this k


def shard_mode(temperature, top_k, top_p, V: int, do_sample: bool = True) -> int:
    """Sampler mode of a vocab-sharded head: 0 greedy, 1 full-vocab sampling, 2 top-k (<= 128)
    (+ top-p); -1 when the configuration does not shard (top-p without top-k, top-k > 128)."""
    tk = int(top_k or 0)
    tp = float(top_p if top_p is not None else 1.0)
    if not do_sample or temperature <= 0:
        return 0
    if (tk <= 0 or tk >= V) and tp >= 1.0:
        return 1
    if 0 < tk <= SHARD_CCAP and tk < V:
        return 2
    return -1


def shard_candidate_shapes(B: int, Vs: int, V: int, mode: int, device) -> list:
    """(shape, dtype) of the tensors ``sample_shard`` returns for a shard of Vs columns — the
    receive buffers of the rank that merges."""
    if torch.device(device).type == "cuda" and not _REF_ON_GPU:
        C = int(ext().sample_shard_chunks(Vs, V))
        if mode == 2:
            return [((B, C * SHARD_CCAP), torch.long), ((B, C), torch.int32)]
        return [((B, C), torch.long)]
    k = min(SHARD_CCAP, Vs) if mode == 2 else 1
    return [((B, k), torch.float32), ((B, k), torch.long)]


def sample_shard(logits, seen, temperature, top_k, top_p, repetition_penalty, rng, v0: int, V: int,
                 do_sample: bool = True):
    """Sampler phase 1 over a vocab shard: ``logits`` [B, Vs] are columns [v0, v0 + Vs) of the
    V-wide rows, ``seen`` the shard's repetition-penalty flags.  Returns the shard's candidate
    tensors (``shard_candidate_shapes``) for ``sample_merge``; the ids in them are global, so the
    merged token is exactly the unsplit sampler's (same processing, same counter-based noise)."""
    mode = shard_mode(temperature, top_k, top_p, V, do_sample)
    assert mode >= 0, "sampling configuration does not shard over the vocabulary"
    if _gpu(logits):
        r = ext().sample_shard(_logits32(logits), seen, float(temperature), int(top_k or 0),
                               float(top_p if top_p is not None else 1.0), float(repetition_penalty),
                               bool(do_sample), rng, int(v0), int(V))
        return tuple(r) if mode == 2 else (r[0],)
    s = logits.float()
    if seen is not None and repetition_penalty != 1.0:     # the processor order of _ref.process_logits
        m = seen.bool()
        s = torch.where(m, torch.where(s < 0, s * repetition_penalty, s / repetition_penalty), s)
    B, Vs = s.shape
    ids = torch.arange(v0, v0 + Vs, device=s.device).expand(B, Vs)
    if mode >= 1 and temperature != 1.0:
        s = s * (1.0 / temperature)
    if mode == 1:
        import numpy as np
        seed, step = (int(v) for v in rng.tolist())
        rows = np.arange(B, dtype=np.uint32)[:, None]
        u = _ref.uniform_hash(seed, rows, step, np.arange(v0, v0 + Vs, dtype=np.uint32)[None, :]).astype(np.float32)
        s = s + torch.from_numpy(-np.log(-np.log(u))).to(s.device)
    if mode <= 1:                                          # best (value, then lower id): argmax = first max
        i = s.argmax(-1, keepdim=True)
        return s.gather(1, i), ids.gather(1, i)
    vals, idx = torch.topk(s, min(SHARD_CCAP, Vs), dim=-1)
    kth = vals[:, min(int(top_k), Vs) - 1:min(int(top_k), Vs)]
    return vals.masked_fill(vals < kth, float("-inf")), ids.gather(1, idx)


def sample_merge(shards, V: int, temperature, top_k, top_p, rng, do_sample: bool = True):
    """Sampler phase 2 over every shard's candidates (``sample_shard`` outputs, in shard order)
    -> tokens [B] (int64): the token the unsplit sampler draws from the whole row."""
    mode = shard_mode(temperature, top_k, top_p, V, do_sample)
    first = shards[0][0]
    if _gpu(first):
        pc = torch.cat([s[0] for s in shards], 1)
        pthr = torch.cat([s[1] for s in shards], 1) if mode == 2 else torch.empty(0, dtype=torch.int32,
                                                                                   device=first.device)
        return ext().sample_merge(pc, pthr, int(V), float(temperature), int(top_k or 0),
                                  float(top_p if top_p is not None else 1.0), bool(do_sample), rng)
    vals = torch.cat([s[0] for s in shards], 1)
    ids = torch.cat([s[1] for s in shards], 1)
    if mode <= 1:
        best = vals.amax(1, keepdim=True)
        big = torch.full_like(ids, torch.iinfo(torch.long).max)
        return torch.where(vals == best, ids, big).amin(1)
    full = torch.full((vals.shape[0], V), float("-inf"), device=vals.device)
    full.scatter_(1, ids, vals)
    seed, step = (int(v) for v in rng.tolist())
    # the shards applied penalty and temperature: the remaining processors are top-k / top-p
    return _ref.sample(full, None, 1.0, top_k, top_p, 1.0, seed, step, True)


def seen_mark(seen, tok, v0: int) -> None:
    """Set the repetition-penalty flag of each row's token in a vocab shard's ``seen`` [B, Vs]
    (tokens outside [v0, v0 + Vs) leave the row unchanged; graph-capturable)."""
    Vs = seen.shape[1]
    j = tok.view(-1, 1) - v0
    inr = (j >= 0) & (j < Vs)
    jc = j.clamp(0, Vs - 1)
    seen.scatter_(1, jc, seen.gather(1, jc) | inr.to(seen.dtype))


def decode_advance(nxt, tok, out, step, pos, seq_lens, rng, inc=None) -> None:
    """Decode-step bookkeeping after sampling: tok = nxt, out[:, step] = nxt, pos += inc,
    seq_lens += inc (``inc``: int32 [B] per-row increments, default 1), rng[1] += 1, step += 1 —
    one launch on the GPU instead of five element-wise ops."""
    if _gpu(nxt):
        ext().decode_advance(nxt, tok, out, step, pos, seq_lens, rng, inc)
        return
    tok.copy_(nxt)
    out.scatter_(1, step.view(1, 1).expand(nxt.shape[0], 1), nxt.view(-1, 1))
    pos.add_(1 if inc is None else inc)
    seq_lens.add_(1 if inc is None else inc)
    rng[1:].add_(1)
    step.add_(1)


FUSE_ADVANCE = os.environ.get("EDGELLM_FUSE_ADVANCE", "1") != "0"


def sample_advance(logits, seen, temperature, top_k, top_p, repetition_penalty, rng, tok, out, step, pos, seq_lens,
                   ctr, do_sample: bool = True):
    """``sample`` then ``decode_advance`` (inc = 1); on the GPU the bookkeeping runs in the
    sampler's last launch (one kernel boundary fewer per decode step).  ``ctr``: int32 [1] zero
    buffer the kernel uses as an arrival counter (it stays zero between calls).  Returns nxt."""
    if _gpu(logits) and FUSE_ADVANCE:
        logits = _logits32(logits)
        nxt = ext().sample_advance(logits, seen, float(temperature), int(top_k or 0),
                                   float(top_p if top_p is not None else 1.0), float(repetition_penalty),
                                   bool(do_sample), rng, tok, out, step, pos, seq_lens, ctr)
        if nxt.numel() > 0 or logits.shape[0] == 0:
            return nxt
    nxt = sample(logits, seen, temperature, top_k, top_p, repetition_penalty, rng, do_sample)
    decode_advance(nxt, tok, out, step, pos, seq_lens, rng)
    return nxt


def max_softmax_prob(logits):
    if _gpu(logits):
        return ext().max_prob(logits.contiguous())
    return _ref.max_softmax_prob(logits)


def embedding(ids, table, out_f32: bool = False):
    """Rows of ``table`` (bf16) for ``ids``; ``out_f32``: as fp32 (exact), e.g. the one split-K slice
    of a first norm deferred into the next GEMV (models.decoder.DecoderLM.embed_tokens)."""
    if _gpu(table):
        return ext().embedding(ids.long().contiguous(), table, out_f32)
    out = _ref.embedding(ids, table)
    return out.float() if out_f32 else out


rope_tables = _ref.rope_tables

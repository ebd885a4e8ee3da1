"""Pure-PyTorch reference implementations of every fused op.

These define the semantics of the HIP kernels in ``ops/csrc`` (each HIP kernel test
compares against the function of the same name here, computed in fp32) and they are
the execution path on CPU (the GPT-2 gRPC plumbing config and all CPU tests).

Reference ops reached through the reference's dependencies are listed in SURVEY.md §2.3
(K1-K13); the comments below name the K# each function covers.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------- norms (K2a/K2b/K8)


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float,
             residual: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """out = rmsnorm(x + residual) * w ; returns (out, x + residual).  fp32 math."""
    # the residual stream is kept in the activation dtype (as HF does): normalise the rounded sum
    res_out = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    h = res_out.float()
    y = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    return y.to(x.dtype), res_out


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], eps: float,
               residual: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    # the residual stream is kept in the activation dtype (as HF does): normalise the rounded sum
    res_out = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    h = res_out.float()
    y = F.layer_norm(h, (h.shape[-1],), weight.float(), None if bias is None else bias.float(), eps)
    return y.to(x.dtype), res_out


def quant_per_token(y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Symmetric per-row int8: scale = max|y|/127, q = round(y/scale)  (K2b epilogue, W8A8)."""
    y = y.float()
    amax = y.abs().amax(-1).clamp_min(1e-8)
    scale = amax / 127.0
    q = torch.round(y / scale[..., None]).clamp_(-127, 127).to(torch.int8)
    return q, scale


def quant_per_group(y: torch.Tensor, group: int = 64) -> Tuple[torch.Tensor, torch.Tensor]:
    """Symmetric int8 with one scale per (row, ``group`` columns); scales laid out
    ``[K/group, Mpad]`` (Mpad = rows rounded up to 16, zero padded) — the decode-GEMV layout."""
    y = y.float()
    M, K = y.shape
    assert K % group == 0
    amax = y.view(M, K // group, group).abs().amax(-1).clamp_min(1e-8)        # [M, G]
    scale = amax / 127.0
    q = torch.round(y.view(M, K // group, group) / scale[..., None]).clamp_(-127, 127).to(torch.int8)
    mpad = (M + 15) // 16 * 16
    s = torch.zeros(K // group, mpad, dtype=torch.float32, device=y.device)
    s[:, :M] = scale.t()
    return q.view(M, K), s


GLU_BLOCK = 16   # gate_up rows packed [gate(16) | up(16)] per 32 rows for the fused decode GLU


def unblock_glu(x: torch.Tensor, block: int = GLU_BLOCK) -> torch.Tensor:
    """Blocked [gate(block) | up(block)] columns -> [gate | up]."""
    M, W = x.shape[:-1], x.shape[-1]
    v = x.reshape(*M, W // (2 * block), 2, block)
    return torch.cat([v[..., 0, :].reshape(*M, W // 2), v[..., 1, :].reshape(*M, W // 2)], -1)


def block_glu_rows(w: torch.Tensor, block: int = GLU_BLOCK) -> torch.Tensor:
    """Rows [gate | up] (2F, ...) -> blocked [gate(block) | up(block)] order (inverse of unblock_glu)."""
    F = w.shape[0] // 2
    g, u = w[:F].reshape(F // block, block, *w.shape[1:]), w[F:].reshape(F // block, block, *w.shape[1:])
    return torch.stack([g, u], 1).reshape(2 * F, *w.shape[1:])


def unblock_glu_rows(w: torch.Tensor, block: int = GLU_BLOCK) -> torch.Tensor:
    """Inverse of block_glu_rows: blocked rows -> [gate | up]."""
    F = w.shape[0] // 2
    v = w.reshape(F // block, 2, block, *w.shape[1:])
    return torch.cat([v[:, 0].reshape(F, *w.shape[1:]), v[:, 1].reshape(F, *w.shape[1:])], 0)


def rms_norm_quant(x, weight, eps, residual=None):
    # the residual stream is kept in the activation dtype (as HF does): normalise the rounded sum
    res_out = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    h = res_out.float()
    y = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    q, s = quant_per_token(y)
    return q, s, res_out


def layer_norm_quant(x, weight, bias, eps, residual=None):
    # the residual stream is kept in the activation dtype (as HF does): normalise the rounded sum
    res_out = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    h = res_out.float()
    y = F.layer_norm(h, (h.shape[-1],), weight.float(), None if bias is None else bias.float(), eps)
    q, s = quant_per_token(y)
    return q, s, res_out


# --------------------------------------------------------------------------- activations (K7)


def silu_mul(x: torch.Tensor) -> torch.Tensor:
    """x = [gate | up] along the last dim -> silu(gate) * up."""
    f = x.shape[-1] // 2
    xf = x.float()
    return (F.silu(xf[..., :f]) * xf[..., f:]).to(x.dtype)


def silu_mul_quant(x: torch.Tensor):
    f = x.shape[-1] // 2
    xf = x.float()
    return quant_per_token(F.silu(xf[..., :f]) * xf[..., f:])


def gelu(x: torch.Tensor, approximate: str = "tanh") -> torch.Tensor:
    return F.gelu(x.float(), approximate=approximate).to(x.dtype)


def gelu_quant(x: torch.Tensor, approximate: str = "tanh"):
    return quant_per_token(F.gelu(x.float(), approximate=approximate))


# --------------------------------------------------------------------------- RoPE + KV write (K4, K6)


def rope_tables(rotary_dim: int, max_pos: int, theta: float, scaling: Optional[dict] = None,
                device=None) -> torch.Tensor:
    """cos/sin table [max_pos, rotary_dim/2, 2] f32, HF "rotate_half" convention,
    with Llama-3 frequency scaling when ``scaling['rope_type'] == 'llama3'``."""
    inv = 1.0 / (theta ** (torch.arange(0, rotary_dim, 2, dtype=torch.float64) / rotary_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling["low_freq_factor"], scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        smooth = (old / wl - lo) / (hi - lo)
        mid = (1 - smooth) * scaled / factor + smooth * scaled
        is_mid = (wl >= hi_wl) & (wl <= lo_wl)
        inv = torch.where(is_mid, mid, scaled)
    elif scaling and scaling.get("rope_type", scaling.get("type")) == "linear":
        inv = inv / scaling["factor"]
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return torch.stack([ang.cos(), ang.sin()], -1).float().to(device)


def _rotate(x: torch.Tensor, cs: torch.Tensor, rotary_dim: int) -> torch.Tensor:
    # x [..., D] f32 ; cs [..., rot/2, 2]
    half = rotary_dim // 2
    x1, x2, rest = x[..., :half], x[..., half:rotary_dim], x[..., rotary_dim:]
    c, s = cs[..., 0], cs[..., 1]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s, rest], -1)


def rope_kv_write(qkv: torch.Tensor, start_pos: torch.Tensor, rope: Optional[torch.Tensor],
                  k_cache: torch.Tensor, v_cache: torch.Tensor,
                  num_heads: int, num_kv_heads: int, head_dim: int, rotary_dim: int,
                  k2: Optional[torch.Tensor] = None, v2: Optional[torch.Tensor] = None, split: int = -1,
                  cpos2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qkv [B*T, (Hq+2Hkv)*D]; token t of sequence b sits at position start_pos[b]+t.
    Rotates q and k (rotate_half on the first ``rotary_dim`` dims), writes k,v into the
    head-major caches ``[B, Hkv, S, D]`` and returns q ``[B, T, Hq, D]``."""
    B = k_cache.shape[0]
    T = qkv.shape[0] // B
    hq, hk, d = num_heads, num_kv_heads, head_dim
    x = qkv.view(B, T, -1).float()
    q = x[..., :hq * d].view(B, T, hq, d)
    k = x[..., hq * d:(hq + hk) * d].view(B, T, hk, d)
    v = x[..., (hq + hk) * d:].view(B, T, hk, d)
    pos = start_pos.long()[:, None] + torch.arange(T, device=qkv.device)[None]  # [B,T]
    if rope is not None and rotary_dim > 0:
        cs = rope[pos][:, :, None]  # [B,T,1,rot/2,2]
        q = _rotate(q, cs, rotary_dim)
        k = _rotate(k, cs, rotary_dim)
    sh = hk if split is None or split < 0 else split
    for b in range(B):
        p = pos[b]
        k_cache[b, :, p] = k[b, :, :sh].transpose(0, 1).to(k_cache.dtype)
        v_cache[b, :, p] = v[b, :, :sh].transpose(0, 1).to(v_cache.dtype)
        if sh < hk:
            p2 = (cpos2.long()[b] if cpos2 is not None else start_pos.long()[b]) + torch.arange(T, device=qkv.device)
            k2[b, :, p2] = k[b, :, sh:].transpose(0, 1).to(k2.dtype)
            v2[b, :, p2] = v[b, :, sh:].transpose(0, 1).to(v2.dtype)
    return q.to(qkv.dtype)


def quant_kv_rows(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """int8 KV cache rows: per-(token, head) symmetric quantisation over the last dim
    (ops/csrc/attn_decode_i8.hip::quant_row16): q = rint(x * 127 / amax), scale = amax / 127."""
    x = x.float()
    amax = x.abs().amax(-1).clamp_min(1e-8)
    q = torch.round(x * (127.0 / amax)[..., None]).clamp(-127, 127).to(torch.int8)
    return q, amax / 127.0


def dequant_kv(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    return q.float() * s[..., None]


def rope_kv_write_i8(qkv: torch.Tensor, start_pos: torch.Tensor, rope: Optional[torch.Tensor],
                     k_cache: torch.Tensor, v_cache: torch.Tensor, k_scale: torch.Tensor, v_scale: torch.Tensor,
                     num_heads: int, num_kv_heads: int, head_dim: int, rotary_dim: int) -> torch.Tensor:
    """rope_kv_write into an int8 cache: the rotated k / v rows (rounded to the activation dtype,
    as the bf16 cache stores them) are quantised per (token, head); returns q [B, T, Hq, D]."""
    B = k_cache.shape[0]
    T = qkv.shape[0] // B
    hq, hk, d = num_heads, num_kv_heads, head_dim
    x = qkv.view(B, T, -1).float()
    q = x[..., :hq * d].view(B, T, hq, d)
    k = x[..., hq * d:(hq + hk) * d].view(B, T, hk, d)
    v = x[..., (hq + hk) * d:].view(B, T, hk, d)
    pos = start_pos.long()[:, None] + torch.arange(T, device=qkv.device)[None]
    if rope is not None and rotary_dim > 0:
        cs = rope[pos][:, :, None]
        q = _rotate(q, cs, rotary_dim)
        k = _rotate(k, cs, rotary_dim)
    kq, ks = quant_kv_rows(k.to(qkv.dtype))
    vq, vs = quant_kv_rows(v.to(qkv.dtype))
    for b in range(B):
        p = pos[b]
        k_cache[b, :, p] = kq[b].transpose(0, 1)
        v_cache[b, :, p] = vq[b].transpose(0, 1)
        k_scale[b, :, p] = ks[b].transpose(0, 1)
        v_scale[b, :, p] = vs[b].transpose(0, 1)
    return q.to(qkv.dtype)


# --------------------------------------------------------------------------- attention (K5, K6)


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                     seq_lens: torch.Tensor, scale: float) -> torch.Tensor:
    """q [B, Hq, D]; caches [B, Hkv, S, D]; attends to positions [0, seq_lens[b])."""
    B, hq, d = q.shape
    hk = k_cache.shape[1]
    g = hq // hk
    out = torch.empty_like(q)
    for b in range(B):
        n = int(seq_lens[b])
        k = k_cache[b, :, :n].float().repeat_interleave(g, 0)  # [Hq, n, D]
        v = v_cache[b, :, :n].float().repeat_interleave(g, 0)
        s = torch.einsum("hd,hnd->hn", q[b].float(), k) * scale
        p = torch.softmax(s, -1)
        out[b] = torch.einsum("hn,hnd->hd", p, v).to(q.dtype)
    return out


def prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                      start_pos: torch.Tensor, scale: float, causal: bool = True) -> torch.Tensor:
    """q [B, T, Hq, D] for positions start_pos[b] .. start_pos[b]+T-1; keys/values come
    from the caches (already written), positions [0, start_pos[b]+T)."""
    B, T, hq, d = q.shape
    hk = k_cache.shape[1]
    g = hq // hk
    out = torch.empty_like(q)
    for b in range(B):
        s0 = int(start_pos[b])
        n = s0 + T
        k = k_cache[b, :, :n].float().repeat_interleave(g, 0)  # [Hq, n, D]
        v = v_cache[b, :, :n].float().repeat_interleave(g, 0)
        s = torch.einsum("thd,hnd->htn", q[b].float(), k) * scale
        if causal:
            qpos = s0 + torch.arange(T, device=q.device)[:, None]
            kpos = torch.arange(n, device=q.device)[None]
            s = s.masked_fill(kpos > qpos, float("-inf"))
        p = torch.softmax(s, -1)
        out[b] = torch.einsum("htn,hnd->thd", p, v).to(q.dtype)
    return out


# --------------------------------------------------------------------------- INT8 GEMM (K11)


def w8a8_linear(qx: torch.Tensor, x_scale: torch.Tensor, qw: torch.Tensor, w_scale: torch.Tensor,
                bias: Optional[torch.Tensor] = None, out_dtype=torch.bfloat16) -> torch.Tensor:
    """out[m,n] = (sum_k qx[m,k]*qw[n,k]) * x_scale[m] * w_scale[n] (+ bias[n]).
    int32 accumulation is exact in fp64 for K < 2^31/127^2.  A 2-D ``x_scale`` [K/64, Mpad] is
    per (token, 64-column group): each group's exact partial sum takes its own scale."""
    if x_scale.dim() == 2:
        M, K = qx.shape
        xs = x_scale[:, :M].t().double().repeat_interleave(64, dim=1)[:, :K]
        acc = (qx.double() * xs) @ qw.double().t()
        out = acc * w_scale.double()[None, :]
        if bias is not None:
            out = out + bias.double()
        return out.to(out_dtype)
    acc = qx.double() @ qw.double().t()
    out = acc * x_scale.double()[:, None] * w_scale.double()[None, :]
    if bias is not None:
        out = out + bias.double()
    return out.to(out_dtype)


# --------------------------------------------------------------------------- sampling (K10)

_M1 = np.uint32(0x85EBCA6B)
_M2 = np.uint32(0xC2B2AE35)


def _mix32(h: np.ndarray) -> np.ndarray:
    h = h ^ (h >> np.uint32(16))
    h = h * _M1
    h = h ^ (h >> np.uint32(13))
    h = h * _M2
    h = h ^ (h >> np.uint32(16))
    return h


def uniform_hash(seed: int, row, step: int, idx) -> np.ndarray:
    """Counter-based uniform in (0,1): identical bit-for-bit in the HIP sampler."""
    with np.errstate(over="ignore"):
        s = np.uint32(seed & 0xFFFFFFFF)
        h = _mix32(np.asarray(row, dtype=np.uint32) * np.uint32(0x9E3779B1) ^ s)
        h = _mix32(h ^ (np.uint32(step & 0xFFFFFFFF) * np.uint32(0x7FEB352D)))
        h = _mix32(h ^ np.asarray(idx, dtype=np.uint32) * np.uint32(0x846CA68B))
    return ((((h >> np.uint32(9)) << np.uint32(1)) | np.uint32(1)).astype(np.float64)) * (1.0 / 16777216.0)


def process_logits(logits: torch.Tensor, seen: Optional[torch.Tensor], temperature: float, top_k: int,
                   top_p: float, repetition_penalty: float) -> torch.Tensor:
    """HF processor order used by ``generate(do_sample=True)``: repetition penalty
    (divide positive / multiply negative scores of already-seen ids) -> temperature ->
    top-k (keep scores >= k-th largest) -> top-p (drop the ascending-sorted prefix whose
    cumulative probability <= 1-top_p, always keep the top token).  Returns processed
    scores with removed entries = -inf.  (combine_model_fp_updated.py:95-105)"""
    s = logits.float().clone()
    if seen is not None and repetition_penalty != 1.0:
        m = seen.bool()
        pen = torch.where(s < 0, s * repetition_penalty, s / repetition_penalty)
        s = torch.where(m, pen, s)
    if temperature > 0 and temperature != 1.0:
        s = s * (1.0 / temperature)  # same f32 product as the HIP sampler
    V = s.shape[-1]
    if top_k and 0 < top_k < V:
        kth = torch.topk(s, top_k, dim=-1).values[..., -1:]
        s = s.masked_fill(s < kth, float("-inf"))
    if top_p is not None and top_p < 1.0:
        srt, idx = torch.sort(s, dim=-1, descending=False)
        cum = torch.softmax(srt, -1).cumsum(-1)
        remove = cum <= (1 - top_p)
        remove[..., -1:] = False
        rm = torch.zeros_like(remove).scatter(-1, idx, remove)
        s = s.masked_fill(rm, float("-inf"))
    return s


def sample(logits: torch.Tensor, seen: Optional[torch.Tensor], temperature: float, top_k: int,
           top_p: float, repetition_penalty: float, seed: int, step: int,
           do_sample: bool = True) -> torch.Tensor:
    """Fused-sampler semantics: HF processing then Gumbel-max with counter-based noise
    (exact sampling from the processed softmax; deterministic given (seed, row, step))."""
    if not do_sample or temperature == 0:
        s = logits.float()
        if seen is not None and repetition_penalty != 1.0:
            m = seen.bool()
            s = torch.where(m, torch.where(s < 0, s * repetition_penalty, s / repetition_penalty), s)
        return s.argmax(-1)
    s = process_logits(logits, seen, temperature, top_k, top_p, repetition_penalty)
    B, V = s.shape
    rows = np.arange(B, dtype=np.uint32)[:, None]
    idx = np.arange(V, dtype=np.uint32)[None, :]
    u = uniform_hash(seed, rows, step, idx).astype(np.float32)
    g = -np.log(-np.log(u))
    g = torch.from_numpy(g).to(s.device)
    return (s + g).argmax(-1)


# --------------------------------------------------------------------------- confidence (K13)


def max_softmax_prob(logits: torch.Tensor) -> torch.Tensor:
    """Per-row max softmax probability = 1 / sum(exp(l - max))  (combine_model_fp_updated.py:76-83)."""
    l = logits.float()
    m = l.amax(-1, keepdim=True)
    return 1.0 / torch.exp(l - m).sum(-1)


# --------------------------------------------------------------------------- embedding (K1)


def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    return F.embedding(ids.long(), table)

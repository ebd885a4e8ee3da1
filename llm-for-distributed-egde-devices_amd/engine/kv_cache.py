"""Preallocated head-major KV cache.

Layout per layer: ``[B, Hkv, S, D]`` (D contiguous, then positions): every (sequence, head) is
one contiguous ``S*D`` run, so
  * decode attention streams a head's keys as one contiguous range (coalesced 1 KiB wave loads),
  * HeadInfer offload moves a head with one contiguous copy (edgellm.offload),
  * a micro-batch / request slot is a contiguous slice along B (``rows``).
Sized up front (no per-token ``torch.cat`` as in HF DynamicCache): with 288 GB of
HBM a Llama-2-7B bf16 cache of 64 sequences x 4096 tokens (128 GB) still fits beside the weights.

``kv_dtype="int8"``: k / v are int8 with one fp32 scale per (token, head) (``ks`` / ``vs``
[L, B, Hkv, S]); decode attention reads D + 4 bytes per row instead of 2 D (1.94x fewer at
D = 128) and the quantising append is fused into the decode attention kernel
(ops/csrc/attn_decode_i8.hip).  Needs head_dim 64 / 128 / 256.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..models.configs import ModelConfig


def resolve_kv_dtype(kv_dtype: str, cfg: ModelConfig, dtype=torch.bfloat16, device=None) -> str:
    """The KV-cache dtype a model can run: int8 needs head_dim 64 / 128 / 256, and on the GPU a
    bf16 model (the int8-KV kernels, attn_decode_i8.hip / kv_quant_append, take bf16 q / k / v);
    otherwise the cache falls back to the model's 16-bit dtype, with a log line."""
    if kv_dtype != "int8":
        return kv_dtype
    why = None
    if cfg.head_dim not in (64, 128, 256):
        why = f"head_dim {cfg.head_dim}"
    elif dtype == torch.float16 and device is not None and torch.device(device).type == "cuda":
        why = "an fp16 model"
    if why is None:
        return "int8"
    from ..utils.log import get_logger
    get_logger("kv_cache").info(f"int8 KV cache not available for {why}: using a 16-bit cache")
    return "bf16"


class KVCache:
    def __init__(self, cfg: ModelConfig, max_batch: int, max_seq: int, first_layer: int = 0,
                 last_layer: Optional[int] = None, dtype=torch.bfloat16, device=None,
                 num_kv_heads: Optional[int] = None, kv_dtype: str = "bf16", zero: bool = True):
        """``zero=False``: uninitialised storage (a scratch cache whose rows a prefill writes in full)."""
        assert kv_dtype in ("bf16", "int8"), kv_dtype
        kv_dtype = resolve_kv_dtype(kv_dtype, cfg, dtype, device)
        self.cfg = cfg
        self.first = first_layer
        self.last = cfg.num_layers if last_layer is None else last_layer
        self.max_batch, self.max_seq = max_batch, max_seq
        hk = cfg.num_kv_heads if num_kv_heads is None else num_kv_heads
        shape = (self.last - self.first, max_batch, hk, max_seq, cfg.head_dim)
        self.quantized = kv_dtype == "int8"
        self.kv_dtype = kv_dtype
        new = torch.zeros if zero else torch.empty
        if self.quantized:
            assert cfg.head_dim in (64, 128, 256), "int8 KV cache needs head_dim 64 / 128 / 256"
            self.k = new(shape, dtype=torch.int8, device=device)
            self.v = new(shape, dtype=torch.int8, device=device)
            self.ks = new(shape[:-1], dtype=torch.float32, device=device)
            self.vs = new(shape[:-1], dtype=torch.float32, device=device)
        else:
            self.k = new(shape, dtype=dtype, device=device)
            self.v = new(shape, dtype=dtype, device=device)

    @staticmethod
    def bytes_per_token(cfg: ModelConfig, dtype_bytes: int = 2) -> int:
        return 2 * cfg.num_layers * cfg.num_kv_heads * cfg.head_dim * dtype_bytes

    def layer(self, i: int):
        return self.k[i - self.first], self.v[i - self.first]

    def layer_scales(self, i: int):
        return self.ks[i - self.first], self.vs[i - self.first]

    def rows(self, r0: int, r1: int) -> "KVView":
        return KVView(self, r0, r1)

    def prefill_scratch(self, B: int, S: int, dtype, device):
        """bf16 (k, v) scratch [B, Hkv, S, D] for int8-cache prefill (rotated new rows + the
        dequantised history), one grow-only buffer per stream shared by every layer: the layers of a
        forward run in stream order, so layer i + 1 rewrites it only after layer i's attention."""
        hk, D = self.k.shape[2], self.k.shape[4]
        n = B * hk * S * D
        key = (torch.cuda.current_stream(device).cuda_stream if torch.device(device).type == "cuda" else 0)
        bufs = self.__dict__.setdefault("_scratch", {})
        buf = bufs.get(key)
        if buf is None or buf.numel() < 2 * n or buf.dtype != dtype or buf.device != torch.device(device):
            buf = bufs[key] = torch.empty(2 * n, dtype=dtype, device=device)
        return buf[:n].view(B, hk, S, D), buf[n:2 * n].view(B, hk, S, D)

    def nbytes(self) -> int:
        n = self.k.numel() * self.k.element_size() * 2
        if self.quantized:
            n += self.ks.numel() * 4 * 2
        return n


class KVView:
    """A contiguous slice of cache rows (one micro-batch / request slot group)."""

    def __init__(self, cache: KVCache, r0: int, r1: int):
        self.cache, self.r0, self.r1 = cache, r0, r1
        self.quantized = getattr(cache, "quantized", False)

    def layer(self, i: int):
        k, v = self.cache.layer(i)
        return k[self.r0:self.r1], v[self.r0:self.r1]

    def layer_scales(self, i: int):
        ks, vs = self.cache.layer_scales(i)
        return ks[self.r0:self.r1], vs[self.r0:self.r1]

    def prefill_scratch(self, B: int, S: int, dtype, device):
        return self.cache.prefill_scratch(B, S, dtype, device)

"""Preallocated head-major KV cache.

Layout per layer: ``[B, Hkv, S, D]`` (D contiguous, then positions): every (sequence, head) is
one contiguous ``S*D`` run, so
  * decode attention streams a head's keys as one contiguous range (coalesced 1 KiB wave loads),
  * HeadInfer offload moves a head with one contiguous copy (edgellm.offload),
  * a micro-batch / request slot is a contiguous slice along B (``rows``).
Sized up front (no per-token ``torch.cat`` as in HF DynamicCache): with 288 GB of
HBM a Llama-2-7B bf16 cache of 64 sequences x 4096 tokens (128 GB) still fits beside the weights.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..models.configs import ModelConfig


class KVCache:
    def __init__(self, cfg: ModelConfig, max_batch: int, max_seq: int, first_layer: int = 0,
                 last_layer: Optional[int] = None, dtype=torch.bfloat16, device=None,
                 num_kv_heads: Optional[int] = None):
        self.cfg = cfg
        self.first = first_layer
        self.last = cfg.num_layers if last_layer is None else last_layer
        self.max_batch, self.max_seq = max_batch, max_seq
        hk = cfg.num_kv_heads if num_kv_heads is None else num_kv_heads
        shape = (self.last - self.first, max_batch, hk, max_seq, cfg.head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)

    @staticmethod
    def bytes_per_token(cfg: ModelConfig, dtype_bytes: int = 2) -> int:
        return 2 * cfg.num_layers * cfg.num_kv_heads * cfg.head_dim * dtype_bytes

    def layer(self, i: int):
        return self.k[i - self.first], self.v[i - self.first]

    def rows(self, r0: int, r1: int) -> "KVView":
        return KVView(self, r0, r1)

    def nbytes(self) -> int:
        return self.k.numel() * self.k.element_size() * 2


class KVView:
    """A contiguous slice of cache rows (one micro-batch / request slot group)."""

    def __init__(self, cache: KVCache, r0: int, r1: int):
        self.cache, self.r0, self.r1 = cache, r0, r1

    def layer(self, i: int):
        k, v = self.cache.layer(i)
        return k[self.r0:self.r1], v[self.r0:self.r1]

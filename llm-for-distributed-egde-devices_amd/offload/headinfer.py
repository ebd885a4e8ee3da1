"""HeadInfer-style head-wise KV offload (Research Papers/headinfer.pdf, Algorithm 1).

Per layer, ``h_on`` KV heads live in HBM; the other ``h_off`` heads live in a pinned host pool.
Attention for an offloaded head needs its whole history on the GPU, so per layer and per chunk
of ``chunk_heads`` heads:

  compute stream                               copy stream (side)
  rope + KV write: resident heads -> HBM cache
                   offloaded heads -> new-row
                   buffer (this layer's parity)  --> D2H write-back of the new rows into the pool
  attention over the resident heads               H2D prefetch of chunk 0 / 1 -> ping-pong buf 0 / 1
  [wait buf j ready] append new rows to buf j,
  attention over chunk j, [record buf j free]  --> prefetch chunk j+2 into buf j (after free)

so the PCIe/xGMI copy of chunk j+1 overlaps the attention of chunk j (ping-pong buffers, events
for every hand-off).  Host-side "generation tags" on each staging buffer assert that a buffer is
only read for the (layer, chunk, history) it was filled for (SURVEY §5.2 race detection);
``EDGELLM_OFFLOAD_SYNC=1`` synchronises after every transfer (debug mode).
Prefill is chunked (``chunk_size`` tokens per pass) to bound activation memory, as in the paper.

Capacity example: Llama-3-8B bf16 KV is 128 KiB/token; with 288 GB of HBM the
cache alone fits ~2M tokens, so offload matters for multi-million-token contexts, large batches
or an explicitly capped ``gpu_kv_budget_heads``.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from .. import ops
from ..engine.kv_cache import KVCache
from ..models.configs import ModelConfig

_SYNC = os.environ.get("EDGELLM_OFFLOAD_SYNC", "0") == "1"


class _View:
    def __init__(self, hi: "HeadInferKV", r0: int, r1: int):
        self.hi, self.r0, self.r1 = hi, r0, r1

    def layer(self, i):
        k, v = self.hi.gpu.layer(i)
        return k[self.r0:self.r1], v[self.r0:self.r1]


class HeadInferKV:
    graph_safe = False   # host-orchestrated transfers: not capturable

    def __init__(self, cfg: ModelConfig, max_batch: int, max_seq: int, h_on: int, device=None, first: int = 0,
                 last: Optional[int] = None, chunk_heads: Optional[int] = None, chunk_size: int = 4096,
                 dtype=torch.bfloat16, stage_budget_bytes: float = 2e9, call_rows: Optional[int] = None):
        """``chunk_heads``: offloaded heads staged per transfer; None = as many as fit
        ``stage_budget_bytes`` across the two ping-pong K/V buffers (the paper stages one head at a
        time to fit a 24 GB card; with 288 GB of HBM larger chunks cut the per-head launches).
        ``call_rows``: most cache rows one forward touches (a pipeline micro-batch); the staging
        and new-row buffers are sized by it instead of by the whole cache (``max_batch``)."""
        hk, D = cfg.num_kv_heads, cfg.head_dim
        assert 0 <= h_on <= hk, "h_on must be within [0, num_kv_heads]"
        self.cfg, self.first = cfg, first
        self.last = cfg.num_layers if last is None else last
        L = self.last - first
        self.h_on, self.h_off = h_on, hk - h_on
        self.max_batch, self.max_seq, self.chunk_size = max_batch, max_seq, chunk_size
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.cuda = self.device.type == "cuda"
        self.gpu = KVCache(cfg, max_batch, max_seq, first, self.last, dtype, device, num_kv_heads=h_on)
        R = self.call_rows = min(max_batch, call_rows or max_batch)
        if chunk_heads is None:
            per_head = 2 * 2 * R * max_seq * D * torch.finfo(dtype).bits // 8   # 2 buffers x (k, v)
            chunk_heads = int(max(1, stage_budget_bytes // max(per_head, 1)))
        self.c = max(1, min(chunk_heads, max(self.h_off, 1)))
        pin = self.cuda
        self.host_k = torch.zeros((L, max_batch, self.h_off, max_seq, D), dtype=dtype, pin_memory=pin)
        self.host_v = torch.zeros_like(self.host_k, pin_memory=pin)
        mk = lambda *s: torch.zeros(*s, dtype=dtype, device=device)  # noqa: E731
        self.stage = [(mk(R, self.c, max_seq, D), mk(R, self.c, max_seq, D)) for _ in range(2)]
        self.new = [(mk(R, self.h_off, chunk_size, D), mk(R, self.h_off, chunk_size, D))
                    for _ in range(2)]
        self.zeros = torch.zeros(max_batch, dtype=torch.int32, device=device)
        if self.cuda:
            self.copy_stream = torch.cuda.Stream(device=self.device)
            self.ev_stage_ready = [torch.cuda.Event() for _ in range(2)]
            self.ev_stage_free = [torch.cuda.Event() for _ in range(2)]
            self.ev_new_free = [torch.cuda.Event() for _ in range(2)]
        self.tags = [None, None]
        self.bytes_h2d = 0
        self.bytes_d2h = 0
        self.transports = {}              # transport name -> copies (offload statistics, tests)
        self.copy_mode = int(os.environ.get("EDGELLM_HEADINFER_COPY_MODE", "0"))   # 0 auto, 1 kernel, 2 dma
        self.attn_hook = self

    # -------------------------------------------------------------- KV-cache interface
    def rows(self, r0: int, r1: int) -> _View:
        return _View(self, r0, r1)

    def layer(self, i):
        return self.gpu.layer(i)

    def gpu_bytes(self) -> int:
        n = self.gpu.nbytes() + sum(t.numel() * t.element_size() for p in self.stage + self.new for t in p)
        return n

    def host_bytes(self) -> int:
        return 2 * self.host_k.numel() * self.host_k.element_size()

    # -------------------------------------------------------------- transfers
    def _copy(self, dst, src):
        t = ops.copy_head_block(dst, src, self.copy_mode)
        self.transports[t] = self.transports.get(t, 0) + 1
        if _SYNC and self.cuda:
            torch.cuda.synchronize()

    def _prefetch(self, buf: int, li: int, r0: int, r1: int, h0: int, cc: int, hist: int):
        sk, sv = self.stage[buf]
        self.tags[buf] = (li, h0, hist, r0, r1)
        if hist == 0:
            if self.cuda:
                self.ev_stage_ready[buf].record(torch.cuda.current_stream())
            return
        if self.cuda:
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_event(self.ev_stage_free[buf])
                self._copy(sk[: r1 - r0, :cc, :hist], self.host_k[li, r0:r1, h0:h0 + cc, :hist])
                self._copy(sv[: r1 - r0, :cc, :hist], self.host_v[li, r0:r1, h0:h0 + cc, :hist])
                self.ev_stage_ready[buf].record(self.copy_stream)
        else:
            self._copy(sk[: r1 - r0, :cc, :hist], self.host_k[li, r0:r1, h0:h0 + cc, :hist])
            self._copy(sv[: r1 - r0, :cc, :hist], self.host_v[li, r0:r1, h0:h0 + cc, :hist])
        self.bytes_h2d += 2 * (r1 - r0) * cc * hist * self.cfg.head_dim * sk.element_size()

    # -------------------------------------------------------------- attention hook
    def attention(self, layer_idx: int, qkv: torch.Tensor, ctx, scale: float, rot: int) -> torch.Tensor:
        cfg = self.cfg
        B, T = ctx.B, ctx.T
        assert T <= self.chunk_size, "prefill must be chunked to <= chunk_size tokens"
        assert B <= self.call_rows, "a forward may touch at most call_rows cache rows"
        hq, hk, D = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
        G = hq // hk
        r0, r1 = ctx.kv.r0, ctx.kv.r1
        li = layer_idx - self.first
        hist = ctx.max_len - T                       # positions already cached (equal lengths)
        par = li % 2
        cs = torch.cuda.current_stream() if self.cuda else None
        if self.cuda:
            cs.wait_event(self.ev_new_free[par])     # write-back of layer li-2 has drained this buffer
        nk = self.new[par][0][:B, :, :T]
        nv = self.new[par][1][:B, :, :T]
        kres, vres = ctx.kv.layer(layer_idx)
        q = ops.rope_kv_write(qkv, ctx.start_pos, ctx.rope if rot else None, kres, vres, hq, hk, D, rot,
                              nk, nv, self.h_on, self.zeros[:B])          # [B, T, Hq, D]
        # write the offloaded heads' new rows back to the host pool (side stream)
        if self.h_off:
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(cs)
                with torch.cuda.stream(self.copy_stream):
                    self.copy_stream.wait_event(ev)
                    self._copy(self.host_k[li, r0:r1, :, hist:hist + T], nk)
                    self._copy(self.host_v[li, r0:r1, :, hist:hist + T], nv)
                    self.ev_new_free[par].record(self.copy_stream)
            else:
                self._copy(self.host_k[li, r0:r1, :, hist:hist + T], nk)
                self._copy(self.host_v[li, r0:r1, :, hist:hist + T], nv)
            self.bytes_d2h += 2 * B * self.h_off * T * D * nk.element_size()
        out = torch.empty(B, T, hq, D, dtype=q.dtype, device=q.device)
        if self.h_on:
            out[:, :, : self.h_on * G] = self._attend(q[:, :, : self.h_on * G], kres, vres, ctx, scale)
        chunks = list(range(0, self.h_off, self.c))
        for j in range(min(2, len(chunks))):
            h0 = chunks[j]
            self._prefetch(j % 2, li, r0, r1, h0, min(self.c, self.h_off - h0), hist)
        for j, h0 in enumerate(chunks):
            buf = j % 2
            cc = min(self.c, self.h_off - h0)
            assert self.tags[buf] == (li, h0, hist, r0, r1), f"stale staging buffer {self.tags[buf]}"
            if self.cuda:
                cs.wait_event(self.ev_stage_ready[buf])
            sk, sv = self.stage[buf]
            sk[:B, :cc, hist:hist + T].copy_(nk[:, h0:h0 + cc])
            sv[:B, :cc, hist:hist + T].copy_(nv[:, h0:h0 + cc])
            qa, qb = (self.h_on + h0) * G, (self.h_on + h0 + cc) * G
            out[:, :, qa:qb] = self._attend(q[:, :, qa:qb], sk[:B, :cc], sv[:B, :cc], ctx, scale)
            if self.cuda:
                self.ev_stage_free[buf].record(cs)
            if j + 2 < len(chunks):
                nh0 = chunks[j + 2]
                self._prefetch(buf, li, r0, r1, nh0, min(self.c, self.h_off - nh0), hist)
        return out.view(B, hq, D) if ctx.mode == "decode" else out

    @staticmethod
    def _attend(q, k, v, ctx, scale):
        if ctx.mode == "decode":
            B, _, h, D = q.shape
            return ops.decode_attention(q[:, 0], k, v, ctx.seq_lens, scale, ctx.max_len).view(B, 1, h, D)
        return ops.prefill_attention(q.contiguous(), k, v, ctx.start_pos, scale, ctx.causal)

    def synchronize(self):
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.copy_stream)


def heads_for_budget(cfg: ModelConfig, max_batch: int, max_seq: int, gpu_kv_budget_bytes: float,
                     layers: Optional[int] = None) -> int:
    """Largest H_on whose resident cache fits the budget (S_on = 2·B·S·D·bytes per head-layer)."""
    layers = layers or cfg.num_layers
    per_head = 2 * max_batch * max_seq * cfg.head_dim * 2 * layers
    return int(max(0, min(cfg.num_kv_heads, gpu_kv_budget_bytes // per_head)))

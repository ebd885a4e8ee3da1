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

``kv_dtype="int8"``: every tier holds int8 K/V with one fp32 scale per (token, head) — the
resident cache (engine.kv_cache int8 layout), the pinned host pool and the staging buffers — so
each decode step moves D + 4 instead of 2 D bytes per (token, head) over PCIe (1.94x fewer at
D = 128).  Decode runs the fused int8 kernel (ops/csrc/attn_decode_i8.hip: RoPE + quantising
append + attention, optionally the per-(token, 64) int8 o-projection input) once on the resident
heads and once per staged chunk, on a gathered QKV slice of those heads; the row the kernel
appended to a staging buffer is written back to the pool from there.  Prefill dequantises the
history into a bf16 scratch exactly like the resident int8 path (models/decoder.py::_forward_kv8)
and quantises the new rows into the cache / staging buffer, so offloaded and resident int8
caches hold the same bytes.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from .. import ops
from ..engine.kv_cache import KVCache, resolve_kv_dtype
from ..models.configs import ModelConfig
from ..models.layers import QAct

_SYNC = os.environ.get("EDGELLM_OFFLOAD_SYNC", "0") == "1"


class _View:
    def __init__(self, hi: "HeadInferKV", r0: int, r1: int):
        self.hi, self.r0, self.r1 = hi, r0, r1

    def layer(self, i):
        k, v = self.hi.gpu.layer(i)
        return k[self.r0:self.r1], v[self.r0:self.r1]

    def layer_scales(self, i):
        ks, vs = self.hi.gpu.layer_scales(i)
        return ks[self.r0:self.r1], vs[self.r0:self.r1]


class HeadInferKV:
    graph_safe = False   # host-orchestrated transfers: not capturable

    def __init__(self, cfg: ModelConfig, max_batch: int, max_seq: int, h_on: int, device=None, first: int = 0,
                 last: Optional[int] = None, chunk_heads: Optional[int] = None, chunk_size: int = 4096,
                 dtype=torch.bfloat16, stage_budget_bytes: float = 2e9, call_rows: Optional[int] = None,
                 kv_dtype: str = "bf16"):
        """``chunk_heads``: offloaded heads staged per transfer; None = as many as fit
        ``stage_budget_bytes`` across the two ping-pong K/V buffers (the paper stages one head at a
        time to fit a 24 GB card; with 288 GB of HBM larger chunks cut the per-head launches).
        ``call_rows``: most cache rows one forward touches (a pipeline micro-batch); the staging
        and new-row buffers are sized by it instead of by the whole cache (``max_batch``).
        ``kv_dtype``: "bf16" or "int8" (int8 K/V + fp32 per-(token, head) scales on every tier)."""
        assert kv_dtype in ("bf16", "int8"), kv_dtype
        kv_dtype = resolve_kv_dtype(kv_dtype, cfg, dtype, device)
        hk, D = cfg.num_kv_heads, cfg.head_dim
        assert 0 <= h_on <= hk, "h_on must be within [0, num_kv_heads]"
        self.cfg, self.first = cfg, first
        self.last = cfg.num_layers if last is None else last
        L = self.last - first
        self.h_on, self.h_off = h_on, hk - h_on
        self.max_batch, self.max_seq, self.chunk_size = max_batch, max_seq, chunk_size
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.cuda = self.device.type == "cuda"
        self.q8 = kv_dtype == "int8"
        self.kv_dtype = kv_dtype
        self.gpu = KVCache(cfg, max_batch, max_seq, first, self.last, dtype, device, num_kv_heads=h_on,
                           kv_dtype=kv_dtype)
        R = self.call_rows = min(max_batch, call_rows or max_batch)
        edt = torch.int8 if self.q8 else dtype
        row_bytes = (D + 4) if self.q8 else D * torch.finfo(dtype).bits // 8
        if chunk_heads is None:
            per_head = 2 * 2 * R * max_seq * row_bytes           # 2 buffers x (k, v)
            chunk_heads = int(max(1, stage_budget_bytes // max(per_head, 1)))
        self.c = max(1, min(chunk_heads, max(self.h_off, 1)))
        pin = self.cuda
        mk = lambda *s, dt=edt: torch.zeros(*s, dtype=dt, device=device)  # noqa: E731
        if self.q8:
            # K and V of a head interleaved as [.., head, {k, v}, S, D] (and their fp32 scales as
            # [.., head, {k, v}, S]) on the host and in the staging buffers: one head-block copy
            # moves both (a [B, 2 c, rows, D] block), halving the per-layer transfers whose fixed
            # cost adds to the PCIe time; k / v are strided views for the kernels
            self.host_kv = torch.zeros((L, max_batch, self.h_off, 2, max_seq, D), dtype=edt, pin_memory=pin)
            self.host_s = torch.zeros((L, max_batch, self.h_off, 2, max_seq), dtype=torch.float32, pin_memory=pin)
            self.host_k, self.host_v = self.host_kv[:, :, :, 0], self.host_kv[:, :, :, 1]
            self.host_ks, self.host_vs = self.host_s[:, :, :, 0], self.host_s[:, :, :, 1]
            self.stage_kv = [mk(R, self.c, 2, max_seq, D) for _ in range(2)]
            self.stage_ss = [mk(R, self.c, 2, max_seq, dt=torch.float32) for _ in range(2)]
            self.stage = [(t[:, :, 0], t[:, :, 1]) for t in self.stage_kv]
            self.stage_s = [(t[:, :, 0], t[:, :, 1]) for t in self.stage_ss]
            self.new = []
        else:
            self.host_k = torch.zeros((L, max_batch, self.h_off, max_seq, D), dtype=edt, pin_memory=pin)
            self.host_v = torch.zeros_like(self.host_k, pin_memory=pin)
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
        self._ahead = None                # (layer, hist, r0, r1) whose chunk 0 is already in flight
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

    def layer_scales(self, i):
        return self.gpu.layer_scales(i)

    def gpu_bytes(self) -> int:
        if self.q8:
            bufs = self.stage_kv + self.stage_ss
            return self.gpu.nbytes() + sum(t.numel() * t.element_size() for t in bufs)
        return self.gpu.nbytes() + sum(t.numel() * t.element_size() for p in self.stage + self.new for t in p)

    def host_bytes(self) -> int:
        if self.q8:
            return self.host_kv.numel() + self.host_s.numel() * 4
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
                self._h2d(buf, li, r0, r1, h0, cc, hist)
                self.ev_stage_ready[buf].record(self.copy_stream)
        else:
            self._h2d(buf, li, r0, r1, h0, cc, hist)
        self.bytes_h2d += 2 * (r1 - r0) * cc * hist * (self.cfg.head_dim * sk.element_size() + (4 if self.q8 else 0))

    def _h2d(self, buf, li, r0, r1, h0, cc, hist):
        if self.q8:                                  # k + v in one block, their scales in another
            B = r1 - r0
            self._copy(self.stage_kv[buf][:B, :cc, :, :hist].flatten(1, 2),
                       self.host_kv[li, r0:r1, h0:h0 + cc, :, :hist].flatten(1, 2))
            self._copy(self.stage_ss[buf][:B, :cc, :, :hist].flatten(1, 2)[..., None],
                       self.host_s[li, r0:r1, h0:h0 + cc, :, :hist].flatten(1, 2)[..., None])
            return
        sk, sv = self.stage[buf]
        self._copy(sk[: r1 - r0, :cc, :hist], self.host_k[li, r0:r1, h0:h0 + cc, :hist])
        self._copy(sv[: r1 - r0, :cc, :hist], self.host_v[li, r0:r1, h0:h0 + cc, :hist])


    def _writeback_q8(self, buf, li, r0, r1, h0, cc, p0, n, cs):
        """int8 rows [p0, p0 + n) that a kernel appended to staging buffer ``buf`` -> the host
        pool (copy stream, after the compute stream's work so far); frees the buffer after."""
        B = r1 - r0

        def go():
            self._copy(self.host_kv[li, r0:r1, h0:h0 + cc, :, p0:p0 + n].flatten(1, 2),
                       self.stage_kv[buf][:B, :cc, :, p0:p0 + n].flatten(1, 2))
            self._copy(self.host_s[li, r0:r1, h0:h0 + cc, :, p0:p0 + n].flatten(1, 2)[..., None],
                       self.stage_ss[buf][:B, :cc, :, p0:p0 + n].flatten(1, 2)[..., None])
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(cs)
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_event(ev)
                go()
                self.ev_stage_free[buf].record(self.copy_stream)
        else:
            go()
        self.bytes_d2h += 2 * B * cc * n * (self.cfg.head_dim + 4)

    # -------------------------------------------------------------- prefetch schedule
    # A layer whose offloaded heads fit ONE staging chunk (the usual case: the 2 GB budget holds 7
    # Llama-3-8B heads at 100K+ tokens) alternates the two buffers by layer, and the next layer's
    # history is issued as soon as this layer's attention is queued: the copy stream then runs
    # H2D(l) -> write-back(l) -> H2D(l+1) back to back while the GEMMs of l and l+1 compute,
    # instead of every layer starting its transfer cold.  Several chunks per layer keep the
    # within-layer ping-pong (buffer = chunk index % 2).
    def _buf(self, li: int, j: int, n: int) -> int:
        return (li + j) % 2 if n == 1 else j % 2

    def _start_prefetch(self, li, r0, r1, hist):
        chunks = list(range(0, self.h_off, self.c))
        ahead = self._ahead == (li, hist, r0, r1)           # issued by the previous layer of this pass
        self._ahead = None
        for j in range(min(2, len(chunks))):
            if ahead and j == 0:
                continue
            h0 = chunks[j]
            self._prefetch(self._buf(li, j, len(chunks)), li, r0, r1, h0, min(self.c, self.h_off - h0), hist)
        return chunks

    def _next_layer_prefetch(self, li, r0, r1, hist):
        if self.h_off and self.c >= self.h_off and li + 1 < self.last - self.first:
            self._prefetch((li + 1) % 2, li + 1, r0, r1, 0, self.h_off, hist)
            self._ahead = (li + 1, hist, r0, r1)

    # -------------------------------------------------------------- attention hook
    def attention(self, layer_idx: int, qkv: torch.Tensor, ctx, scale: float, rot: int, quant_o: bool = False):
        """Attention of one layer over resident + offloaded heads.  Returns bf16 [B, Hq, D]
        (decode) / [B, T, Hq, D] (prefill), or — int8 cache, decode, ``quant_o`` — a ``QAct``
        with the per-(token, 64) int8 o-projection input."""
        if self.q8:
            return self._attention_q8(layer_idx, qkv, ctx, scale, rot, quant_o)
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
        chunks = self._start_prefetch(li, r0, r1, hist)
        for j, h0 in enumerate(chunks):
            buf = self._buf(li, j, len(chunks))
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
        self._next_layer_prefetch(li, r0, r1, hist)
        return out.view(B, hq, D) if ctx.mode == "decode" else out

    def _attention_q8(self, layer_idx: int, qkv: torch.Tensor, ctx, scale: float, rot: int, quant_o: bool):
        cfg = self.cfg
        B, T = ctx.B, ctx.T
        assert T <= self.chunk_size, "prefill must be chunked to <= chunk_size tokens"
        assert B <= self.call_rows, "a forward may touch at most call_rows cache rows"
        hq, hk, D = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
        G = hq // hk
        r0, r1 = ctx.kv.r0, ctx.kv.r1
        li = layer_idx - self.first
        hist = ctx.max_len - T                       # positions already cached (equal lengths)
        cs = torch.cuda.current_stream() if self.cuda else None
        kres, vres = ctx.kv.layer(layer_idx)
        ksr, vsr = ctx.kv.layer_scales(layer_idx)
        rope = ctx.rope if rot else None
        chunks = self._start_prefetch(li, r0, r1, hist)
        if ctx.mode == "decode":
            x = qkv.view(B, -1)

            def sub(h0, n):      # QKV columns of kv heads [h0, h0 + n): their q group, k and v
                return torch.cat([x[:, h0 * G * D:(h0 + n) * G * D], x[:, (hq + h0) * D:(hq + h0 + n) * D],
                                  x[:, (hq + hk + h0) * D:(hq + hk + h0 + n) * D]], 1)
            if quant_o:
                oq = torch.empty(B, hq * D, dtype=torch.int8, device=qkv.device)
                osc = torch.empty(hq * D // 64, (B + 15) // 16 * 16, dtype=torch.float32, device=qkv.device)
            else:
                out = torch.empty(B, hq, D, dtype=qkv.dtype, device=qkv.device)

            def attend(h0, n, kc, vc, ksc, vsc):
                o, s = ops.decode_attention_fused_i8(sub(h0, n), ctx.start_pos, rope, kc, vc, ksc, vsc, ctx.seq_lens,
                                                     n * G, scale, ctx.max_len, rot, quant_o)
                qa, qb = h0 * G, (h0 + n) * G
                if quant_o:
                    oq[:, qa * D:qb * D] = o
                    osc[qa * D // 64:qb * D // 64] = s
                else:
                    out[:, qa:qb] = o
            if self.h_on:
                attend(0, self.h_on, kres, vres, ksr, vsr)
            for j, h0 in enumerate(chunks):
                buf = self._buf(li, j, len(chunks))
                cc = min(self.c, self.h_off - h0)
                assert self.tags[buf] == (li, h0, hist, r0, r1), f"stale staging buffer {self.tags[buf]}"
                if self.cuda:
                    cs.wait_event(self.ev_stage_ready[buf])
                (sk, sv), (sks, svs) = self.stage[buf], self.stage_s[buf]
                attend(self.h_on + h0, cc, sk[:B, :cc], sv[:B, :cc], sks[:B, :cc], svs[:B, :cc])
                self._writeback_q8(buf, li, r0, r1, h0, cc, hist, 1, cs)
                if j + 2 < len(chunks):
                    nh0 = chunks[j + 2]
                    self._prefetch(buf, li, r0, r1, nh0, min(self.c, self.h_off - nh0), hist)
            self._next_layer_prefetch(li, r0, r1, hist)
            return QAct(oq, osc) if quant_o else out
        # prefill chunk: bf16 scratch = dequantised history + the rotated new rows (as the
        # resident int8 path); new rows are quantised into the resident cache / staging buffer
        kb = torch.empty(B, hk, hist + T, D, dtype=qkv.dtype, device=qkv.device)
        vb = torch.empty_like(kb)
        q = ops.rope_kv_write(qkv, ctx.start_pos, rope, kb, vb, hq, hk, D, rot)      # [B, T, Hq, D]
        out = torch.empty(B, T, hq, D, dtype=q.dtype, device=q.device)

        def fill(a, n, kc, vc, ksc, vsc):
            if hist > 0:
                kb[:, a:a + n, :hist] = ops._ref.dequant_kv(kc[:, :, :hist], ksc[:, :, :hist]).to(kb.dtype)
                vb[:, a:a + n, :hist] = ops._ref.dequant_kv(vc[:, :, :hist], vsc[:, :, :hist]).to(vb.dtype)
            ops.kv_quant_append(kb[:, a:a + n], ctx.start_pos, T, kc, ksc)
            ops.kv_quant_append(vb[:, a:a + n], ctx.start_pos, T, vc, vsc)
            out[:, :, a * G:(a + n) * G] = ops.prefill_attention(q[:, :, a * G:(a + n) * G].contiguous(),
                                                                 kb[:, a:a + n], vb[:, a:a + n], ctx.start_pos,
                                                                 scale, ctx.causal)
        if self.h_on:
            fill(0, self.h_on, kres, vres, ksr, vsr)
        for j, h0 in enumerate(chunks):
            buf = self._buf(li, j, len(chunks))
            cc = min(self.c, self.h_off - h0)
            assert self.tags[buf] == (li, h0, hist, r0, r1), f"stale staging buffer {self.tags[buf]}"
            if self.cuda:
                cs.wait_event(self.ev_stage_ready[buf])
            (sk, sv), (sks, svs) = self.stage[buf], self.stage_s[buf]
            fill(self.h_on + h0, cc, sk[:B, :cc], sv[:B, :cc], sks[:B, :cc], svs[:B, :cc])
            self._writeback_q8(buf, li, r0, r1, h0, cc, hist, T, cs)
            if j + 2 < len(chunks):
                nh0 = chunks[j + 2]
                self._prefetch(buf, li, r0, r1, nh0, min(self.c, self.h_off - nh0), hist)
        self._next_layer_prefetch(li, r0, r1, hist)
        return out

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

"""In-process layer split across the GPUs of one agent's device group.

This is the direct counterpart of the reference's only multi-device mechanism, Hugging Face
``device_map="auto"`` (Code/Base Models/Llama_bf16_updated.py:31,
combine_model_fp_updated.py:40, Code/Quantised Models/models_quant_updated.py:36): accelerate
places whole decoder layers on the visible GPUs and hops the hidden state between them with
``tensor.to(next_device)``.  ``SplitLM`` does the same for an edgellm model — layers
[b[s], b[s+1]) live on device s (balanced partition, parallel/partition.py), each stage keeps
its own KV-cache slice on its own device, and the hidden state crosses xGMI as a peer copy
between stages — so every CLI (evaluate / combine / serve) can run a model that is split over
an agent's ``gpus:`` group (``agents[].gpus``) or over ``parallel.pp_size`` devices.

It exposes the DecoderLM / KVCache interfaces the Generator uses, so prefill, sampling, EOS
handling and both TPS definitions are unchanged.  Decode runs eagerly (one HIP graph cannot
span devices); the multi-process RCCL pipeline (parallel/pipeline.py) is the throughput path.
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional, Sequence

import torch
import torch.nn as nn

from ..engine.kv_cache import KVCache
from ..models.decoder import AttnCtx, DecoderLM
from ..models.layers import PartialSum
from .partition import partition_model


class SplitKV:
    """Per-stage KV caches (each on its stage's device) behind the KVCache interface."""

    def __init__(self, caches: Sequence[KVCache], bounds: Sequence[int]):
        self.caches, self.bounds = list(caches), list(bounds)
        self.max_batch, self.max_seq = caches[0].max_batch, caches[0].max_seq
        self.quantized = caches[0].quantized
        self._owner = {}
        for s, c in enumerate(self.caches):
            for i in range(self.bounds[s], self.bounds[s + 1]):
                self._owner[i] = c

    def layer(self, i: int):
        return self._owner[i].layer(i)

    def layer_scales(self, i: int):
        return self._owner[i].layer_scales(i)

    def rows(self, r0: int, r1: int) -> "_SplitView":
        return _SplitView(self, r0, r1)

    def nbytes(self) -> int:
        return sum(c.nbytes() for c in self.caches)


class _SplitView:
    def __init__(self, kv: SplitKV, r0: int, r1: int):
        self.kv, self.r0, self.r1 = kv, r0, r1
        self.quantized = kv.quantized

    def layer(self, i: int):
        k, v = self.kv.layer(i)
        return k[self.r0:self.r1], v[self.r0:self.r1]

    def layer_scales(self, i: int):
        ks, vs = self.kv.layer_scales(i)
        return ks[self.r0:self.r1], vs[self.r0:self.r1]


class SplitLM(nn.Module):
    """A DecoderLM whose layers are spread over ``devices`` (contiguous blocks, in order)."""

    graph_safe = False      # kernels on several devices: decode runs eagerly

    def __init__(self, model: DecoderLM, devices: Sequence[torch.device], bounds: Optional[Sequence[int]] = None):
        super().__init__()
        assert model.has_embed and model.has_head, "split a full model"
        devices = [torch.device(d) for d in devices]
        cfg = model.cfg
        P = len(devices)
        if bounds is None:
            wb = 1.0 if any(getattr(m, "takes_quantized_input", False) for m in model.modules()) else 2.0
            bounds = partition_model(cfg, P, "balanced", weight_bytes=wb)
        assert len(bounds) == P + 1 and bounds[0] == 0 and bounds[-1] == cfg.num_layers
        self.cfg, self.dtype = cfg, model.dtype
        self.devices, self.bounds = devices, list(bounds)
        self.first, self.last = 0, cfg.num_layers
        self.has_embed = self.has_head = True
        self.inner = model
        with torch.no_grad():
            model.embed.data = model.embed.data.to(devices[0])
            if model.pos_embed is not None:
                model.pos_embed.data = model.pos_embed.data.to(devices[0])
            for s in range(P):
                for layer in model.layers[bounds[s]:bounds[s + 1]]:
                    layer.to(devices[s])
            model.final_norm.to(devices[-1])
            if model.lm_head is not None:
                model.lm_head.to(devices[-1])
        self._tied = model.lm_head is None
        self._head_embed = model.embed.data.to(devices[-1]) if self._tied and P > 1 else None
        self._ropes = {}

    # ------------------------------------------------------------------ DecoderLM interface
    @property
    def device(self):
        return self.devices[0]

    def rope_table(self, device=None):
        return self.inner.rope_table(device or self.devices[0])

    def make_kv(self, max_batch: int, max_seq: int, kv_dtype: str = "bf16") -> SplitKV:
        caches = [KVCache(self.cfg, max_batch, max_seq, self.bounds[s], self.bounds[s + 1], self.dtype, d,
                          kv_dtype=kv_dtype) for s, d in enumerate(self.devices)]
        return SplitKV(caches, self.bounds)

    def _ctx_on(self, ctx: AttnCtx, dev: torch.device) -> AttnCtx:
        if ctx.start_pos.device == dev:
            return ctx
        rope = None
        if ctx.rope is not None:
            rope = self._ropes.get(dev)
            if rope is None:
                rope = self._ropes[dev] = ctx.rope.to(dev)
        last = ctx.last_pos.to(dev) if ctx.last_pos is not None else None
        return dataclasses.replace(ctx, start_pos=ctx.start_pos.to(dev), seq_lens=ctx.seq_lens.to(dev), rope=rope,
                                   last_pos=last)

    @torch.no_grad()
    def forward(self, ids: Optional[torch.Tensor], ctx: AttnCtx, hidden: Optional[torch.Tensor] = None,
                logits: str = "last"):
        m = self.inner
        x = m.embed_tokens(ids.to(self.devices[0]), ctx.start_pos) if hidden is None else hidden
        residual = None
        for s, dev in enumerate(self.devices):
            c = self._ctx_on(ctx, dev)
            xd = x.parts.device if isinstance(x, PartialSum) else x.device   # split-K slices (o / down)
            if xd != dev:                                    # the inter-stage hop (xGMI peer copy)
                if isinstance(x, PartialSum):
                    x = x.materialize()
                x = x.to(dev, non_blocking=True)
                residual = residual.to(dev, non_blocking=True) if residual is not None else None
            for layer in m.layers[self.bounds[s]:self.bounds[s + 1]]:
                x, residual = layer(x, residual, c)
        c = self._ctx_on(ctx, self.devices[-1])
        if self._head_embed is not None:
            if isinstance(x, PartialSum):
                x = x.materialize()
            if logits == "last" and c.T > 1:
                idx = c.last_rows(x.device)
                x = x.index_select(0, idx)
                residual = residual.index_select(0, idx) if residual is not None else None
            h, _ = m.final_norm(x, residual)
            out = torch.nn.functional.linear(h, self._head_embed)
        else:
            out = m.head(x, residual, c, logits)
        return out.to(self.devices[0])


def split_model(model: DecoderLM, devices: Sequence, bounds: Optional[Sequence[int]] = None):
    """``model`` itself on one device; a SplitLM over several."""
    devices = [torch.device(d) for d in devices]
    if len(devices) <= 1:
        return model.to(devices[0]) if devices else model
    return SplitLM(model, devices, bounds)


def agent_devices(gpus: Optional[List[int]], fallback: torch.device, pp_size: int = 1) -> List[torch.device]:
    """An agent's device group: its ``gpus:`` list (YAML agents[].gpus), else ``pp_size``
    consecutive devices starting at ``fallback`` (CPU stays one device)."""
    if gpus:
        if not torch.cuda.is_available():
            return [torch.device("cpu")]
        n = torch.cuda.device_count()
        if max(int(g) for g in gpus) >= n:
            from ..utils.log import get_logger
            get_logger("split").warning(f"gpus {list(gpus)} on a {n}-GPU host: folded modulo {n}")
        out: List[torch.device] = []
        for g in gpus:                       # fold onto the visible GPUs, drop repeats in order
            d = torch.device("cuda", int(g) % n)
            if d not in out:
                out.append(d)
        return out
    if pp_size > 1 and fallback.type == "cuda":
        n = torch.cuda.device_count()
        return [torch.device("cuda", ((fallback.index or 0) + i) % n) for i in range(pp_size)]
    if pp_size > 1:                 # CPU: the same stage plumbing, every stage on the host
        return [fallback] * pp_size
    return [fallback]

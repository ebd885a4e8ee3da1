"""LM head split by vocabulary over the pipeline's ranks.

The reference's layer split (accelerate ``device_map="auto"``, Code/Base Models/Llama_bf16_updated.py:31)
leaves the whole LM head — the largest single weight, 262 MB bf16 on Llama-2-7B, plus the sampler —
on the last device, so the last stage is the slowest and sets every stage's tick: at 8 stages of 4
layers the modelled max / mean stage cost is 1.11 (parallel/partition.py).  Here every rank holds
rows [v0, v1) of the head (``shard_bounds``): the last stage hands its final-normed hidden rows to
every rank, each rank computes its logits slice and the sampler's phase 1 over it (candidate lists
with GLOBAL token ids: ops.sample_shard), and rank 0 merges the lists (ops.sample_merge) — the
two-phase fused sampler run over one row, so the sampled token equals the unsplit model's (same
processor order, same counter-based noise per global id).  Rank 0 then feeds the token straight to
its embedding and sends it to the other ranks, which mark it in their shard of the
repetition-penalty flags.  Head cost per stage becomes 1/P of the head; the pipeline needs one more
micro-batch group in flight (``PipelineStage(vocab_split=True)``).
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import nn

from .. import ops
from ..models.configs import ModelConfig
from ..models.layers import Linear


def shard_bounds(V: int, P: int, align: int = 64) -> List[int]:
    """Vocab bounds [b_0 = 0, ..., b_P = V] of P shards: equal ``align``-multiples, the last one
    shorter; every shard non-empty."""
    per = -(-V // P)
    per = -(-per // align) * align
    b = [min(V, r * per) for r in range(P + 1)]
    b[-1] = V
    assert all(b[r + 1] > b[r] for r in range(P)), f"vocab {V} too small for {P} shards of {per}"
    return b


class HeadShard(nn.Module):
    """Rows [v0, v1) of the LM head (+ bias) and the sampler phase 1 over them."""

    def __init__(self, weight: torch.Tensor, bias: Optional[torch.Tensor], v0: int, V: int):
        super().__init__()
        Vs, H = weight.shape
        self.v0, self.v1, self.V = int(v0), int(v0) + Vs, int(V)
        self.proj = Linear(H, Vs, bias is not None, weight.dtype, weight.device)
        with torch.no_grad():
            self.proj.weight.copy_(weight)
            if bias is not None:
                self.proj.bias.copy_(bias)

    @property
    def Vs(self) -> int:
        return self.v1 - self.v0

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        return self.proj(h)

    def candidates(self, h: torch.Tensor, seen: torch.Tensor, sp, rng: torch.Tensor):
        """Phase-1 candidate tensors of this shard for the final-normed rows ``h`` [b, H]."""
        return ops.sample_shard(self.logits(h), seen, sp.temperature, sp.top_k, sp.top_p, sp.repetition_penalty,
                                rng, self.v0, self.V, sp.do_sample)


@torch.no_grad()
def build_head_shard(cfg: ModelConfig, rank: int, world: int, model=None, seed: Optional[int] = 0,
                     dtype=torch.bfloat16, device=None, full_weight: Optional[torch.Tensor] = None,
                     full_bias: Optional[torch.Tensor] = None, checkpoint: Optional[str] = None) -> HeadShard:
    """Rank ``rank``'s head shard.  The weight comes from ``full_weight`` / ``full_bias``, else the
    shard's rows of an edgellm INT8 ``checkpoint`` (quant.checkpoint.load_head_rows), else from
    ``model`` when it holds the (bf16) head, else it is the random-init head of ``seed``
    (models.decoder.random_head_weight: bit-identical to the unsplit model's)."""
    b = shard_bounds(cfg.vocab_size, world)
    v0, v1 = b[rank], b[rank + 1]
    if checkpoint is not None and full_weight is None:
        from ..quant.checkpoint import load_head_rows
        w, bias = load_head_rows(checkpoint, v0, v1, device, dtype)
        return HeadShard(w.contiguous(), bias, v0, cfg.vocab_size)
    if full_weight is None and model is not None and getattr(model, "has_head", False):
        lm = model.lm_head
        assert lm is None or not getattr(lm, "takes_quantized_input", False), "vocab split: 16-bit LM head only"
        full_weight = model.head_weight()
        full_bias = lm.bias if lm is not None else None
    if full_weight is None:
        from ..models.decoder import random_head_weight
        full_weight = random_head_weight(cfg, seed if seed is not None else 0, dtype, device)
        full_bias = torch.zeros(cfg.vocab_size, dtype=dtype, device=device) if cfg.lm_head_bias else None
    w = full_weight[v0:v1].detach().to(dtype=dtype, device=device).contiguous()
    bias = full_bias[v0:v1].detach().to(dtype=dtype, device=device).contiguous() if full_bias is not None else None
    return HeadShard(w, bias, v0, cfg.vocab_size)


@torch.no_grad()
def shard_from_last_stage(model, cfg: ModelConfig, rank: int, world: int, group=None, ranks=None,
                          device=None) -> HeadShard:
    """Every pipeline rank's head shard from the stage that holds the head (the last): it sends
    each other rank its rows once, over the group's P2P path, so the split works for any weight
    source (random init, HF checkpoint, int8 checkpoint) without a rank re-reading the head.
    Every member of the group must call this, in any order."""
    import torch.distributed as dist
    b = shard_bounds(cfg.vocab_size, world)
    v0, v1 = b[rank], b[rank + 1]
    granks = list(ranks) if ranks is not None else list(range(world))
    nccl = dist.is_initialized() and dist.get_backend(group) == "nccl"
    dev = torch.device(device) if device is not None else model.device
    cdev = dev if nccl else torch.device("cpu")
    dtype = model.dtype
    if rank == world - 1:
        lm = model.lm_head
        assert lm is None or not getattr(lm, "takes_quantized_input", False), "vocab split: 16-bit LM head only"
        W = model.head_weight()
        bias = lm.bias if lm is not None else None
        for r in range(world - 1):
            dist.send(W[b[r]:b[r + 1]].contiguous().to(cdev), granks[r], group=group)
            if bias is not None:
                dist.send(bias[b[r]:b[r + 1]].contiguous().to(cdev), granks[r], group=group)
        return HeadShard(W[v0:v1].contiguous(), bias[v0:v1].contiguous() if bias is not None else None, v0,
                         cfg.vocab_size)
    w = torch.empty(v1 - v0, cfg.hidden_size, dtype=dtype, device=cdev)
    dist.recv(w, granks[-1], group=group)
    bias = None
    if cfg.lm_head_bias:
        bias = torch.empty(v1 - v0, dtype=dtype, device=cdev)
        dist.recv(bias, granks[-1], group=group)
    return HeadShard(w.to(dev), bias.to(dev) if bias is not None else None, v0, cfg.vocab_size)

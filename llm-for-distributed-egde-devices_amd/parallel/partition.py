"""Layer partitioner for the pipeline (replaces accelerate's ``device_map="auto"`` split,
Code/Base Models/Llama_bf16_updated.py:31 — SURVEY §2.4).

Cost model = bytes streamed per decode step (decode is HBM-bound): every decoder layer costs
its weight bytes, the last stage also pays for the LM head (bf16 by default) and the first
stage for the embedding gather (negligible).  The partition minimises the most expensive stage
over all contiguous splits (exact DP, O(P * L^2)), i.e. the pipeline's tick time.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from ..models.configs import ModelConfig


def layer_costs(cfg: ModelConfig, weight_bytes: float = 1.0, head_bytes: float = 2.0,
                head_cost_layers: Optional[float] = None) -> Tuple[List[float], float]:
    """Per-layer costs and the last stage's extra (LM head + sampler).  By default both are bytes
    streamed per step; ``head_cost_layers`` instead prices the head in measured decoder-layer
    times (MI355X W8A8 decode at 64 rows: a layer ~132 us per lane, bf16 head GEMM + fused
    sampler ~80 us, so 0.6 — bytes alone would call the 262 MB bf16 head 1.3 layers)."""
    per = cfg.layer_bytes(weight_bytes)
    if head_cost_layers is not None:
        return [per] * cfg.num_layers, head_cost_layers * per
    head = head_bytes * cfg.hidden_size * cfg.vocab_size
    return [per] * cfg.num_layers, head


def balanced_partition(costs: Sequence[float], stages: int, head_cost: float = 0.0,
                       embed_cost: float = 0.0) -> List[int]:
    """Boundaries b[0]=0 < b[1] < ... < b[P]=L minimising max stage cost."""
    L = len(costs)
    assert 1 <= stages <= L, "need at least one layer per stage"
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)

    def cost(s, a, b):
        c = pre[b] - pre[a]
        if s == 0:
            c += embed_cost
        if s == stages - 1:
            c += head_cost
        return c

    INF = float("inf")
    best = [[INF] * (L + 1) for _ in range(stages + 1)]
    arg = [[0] * (L + 1) for _ in range(stages + 1)]
    best[0][0] = 0.0
    for s in range(1, stages + 1):
        for b in range(s, L - (stages - s) + 1):
            for a in range(s - 1, b):
                if best[s - 1][a] == INF:
                    continue
                v = max(best[s - 1][a], cost(s - 1, a, b))
                if v < best[s][b]:
                    best[s][b], arg[s][b] = v, a
    bounds = [L]
    b = L
    for s in range(stages, 0, -1):
        b = arg[s][b]
        bounds.append(b)
    return bounds[::-1]


def uniform_partition(L: int, stages: int) -> List[int]:
    return [round(i * L / stages) for i in range(stages + 1)]


def partition_model(cfg: ModelConfig, stages: int, mode: str = "balanced", weight_bytes: float = 1.0,
                    head_bytes: float = 2.0, explicit: Optional[str] = None,
                    head_cost_layers: Optional[float] = None) -> List[int]:
    """mode: balanced | uniform | explicit ("8,8,8,8" layers per stage)."""
    if explicit or mode not in ("balanced", "uniform"):
        spec = explicit or mode
        counts = [int(x) for x in spec.split(",")]
        assert len(counts) == stages and sum(counts) == cfg.num_layers, spec
        out = [0]
        for c in counts:
            out.append(out[-1] + c)
        return out
    if mode == "uniform":
        return uniform_partition(cfg.num_layers, stages)
    costs, head = layer_costs(cfg, weight_bytes, head_bytes, head_cost_layers)
    return balanced_partition(costs, stages, head)


def stage_costs(cfg: ModelConfig, bounds: Sequence[int], weight_bytes: float = 1.0, head_bytes: float = 2.0,
                head_cost_layers: Optional[float] = None):
    costs, head = layer_costs(cfg, weight_bytes, head_bytes, head_cost_layers)
    out = []
    for s in range(len(bounds) - 1):
        c = sum(costs[bounds[s]:bounds[s + 1]])
        if s == len(bounds) - 2:
            c += head
        out.append(c)
    return out

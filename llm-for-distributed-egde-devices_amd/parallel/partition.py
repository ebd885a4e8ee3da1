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
                       embed_cost: float = 0.0, stage_extra: Optional[Sequence[float]] = None) -> List[int]:
    """Boundaries b[0]=0 < b[1] < ... < b[P]=L minimising max stage cost (``stage_extra[s]``: a
    fixed cost of stage s on top of its layers, e.g. its share of a vocab-split LM head)."""
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
        if stage_extra is not None:
            c += stage_extra[s]
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


# decode-time model of one half-layer unit on MI355X (us), calibrated on the 256-row W8A8 Llama-2-7B
# bench step (profiles/rocprof_bench_default_r3_final.md): projections stream their weights at the
# measured 256-row decode GEMM rate, attention its KV bytes at the measured attention rate, plus a
# fixed per-half cost (RMSNorm launch + kernel boundaries); the head is its GEMM + sampler + norm.
GEMM_BYTES_PER_US = 2.15e6
ATTN_BYTES_PER_US = 5.9e6
HALF_FIXED_US = 8.0
HEAD_BYTES_PER_US = 3.2e6
HEAD_FIXED_US = 35.0
# vocab-split head (parallel/vocab_head.py): per stage its rows of the head GEMM + the sampler's
# phase 1 over them + the penalty-flag update; rank 0 the merge (phase 2 + bookkeeping); the last
# stage the final norm
SHARD_FIXED_US = 12.0
MERGE_US = 10.0
FINAL_NORM_US = 4.0


def decode_unit_costs(cfg: ModelConfig, rows: int = 256, ctx: int = 160, weight_bytes: float = 1.0,
                      kv_bytes: float = 2.0, head_bytes: float = 2.0) -> Tuple[List[float], float]:
    """Per half-layer unit costs (unit 2 i = layer i's norm1 + attention + o, 2 i + 1 = norm2 +
    MLP) and the head's, in us per decode step of ``rows`` sequences at ``ctx`` cached tokens.
    The attention half carries the KV stream, so at the bench's 256 x ~160 tokens it is about twice
    the MLP half: whole layers (0.5 layer of head on the last stage) cannot balance 8 stages better
    than max / mean 1.11, half layers can."""
    H, I = cfg.hidden_size, cfg.intermediate_size
    w_attn = (cfg.qkv_size * H + H * cfg.q_size) * weight_bytes
    w_mlp = ((2 if cfg.is_glu else 1) * I * H + I * H) * weight_bytes
    kv = 2.0 * rows * ctx * cfg.num_kv_heads * cfg.head_dim * kv_bytes
    attn = w_attn / GEMM_BYTES_PER_US + kv / ATTN_BYTES_PER_US + HALF_FIXED_US
    mlp = w_mlp / GEMM_BYTES_PER_US + HALF_FIXED_US
    head = H * cfg.vocab_size * head_bytes / HEAD_BYTES_PER_US + HEAD_FIXED_US
    return [attn, mlp] * cfg.num_layers, head


def head_split_extra(cfg: ModelConfig, stages: int, head_bytes: float = 2.0) -> List[float]:
    """Per-stage cost (us) of an LM head split by vocabulary over ``stages`` ranks."""
    shard = cfg.hidden_size * cfg.vocab_size * head_bytes / stages / HEAD_BYTES_PER_US + SHARD_FIXED_US
    extra = [shard] * stages
    extra[0] += MERGE_US
    extra[-1] += FINAL_NORM_US
    return extra


def partition_units(cfg: ModelConfig, stages: int, rows: int = 256, ctx: int = 160, weight_bytes: float = 1.0,
                    kv_bytes: float = 2.0, head_bytes: float = 2.0, head_split: bool = False) -> List[int]:
    """Balanced stage boundaries in half-layer units (``DecoderLM.from_units``): a boundary may fall
    between a layer's attention and MLP halves.  Sequential-residual models only; parallel-residual
    ones (Phi-2, Pythia) get whole-layer boundaries (their units in pairs).  ``head_split``: the LM
    head is split by vocabulary over every stage (``head_split_extra``) instead of sitting on the last."""
    costs, head = decode_unit_costs(cfg, rows, ctx, weight_bytes, kv_bytes, head_bytes)
    extra = head_split_extra(cfg, stages, head_bytes) if head_split and stages > 1 else None
    head = 0.0 if extra is not None else head
    if cfg.parallel_residual:
        layer = [costs[2 * i] + costs[2 * i + 1] for i in range(cfg.num_layers)]
        return [2 * b for b in balanced_partition(layer, stages, head, stage_extra=extra)]
    return balanced_partition(costs, stages, head, stage_extra=extra)


def unit_stage_costs(cfg: ModelConfig, bounds: Sequence[int], head_split: bool = False, **kw) -> List[float]:
    """Modelled per-stage cost (us) of unit bounds (``partition_units``)."""
    costs, head = decode_unit_costs(cfg, **kw)
    P = len(bounds) - 1
    out = [sum(costs[bounds[s]:bounds[s + 1]]) for s in range(P)]
    if head_split and P > 1:
        for s, e in enumerate(head_split_extra(cfg, P, kw.get("head_bytes", 2.0))):
            out[s] += e
    else:
        out[-1] += head
    return out


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

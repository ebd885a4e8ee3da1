"""Multi-GPU leg of bench.py: pipeline of N stages (one per GPU), N x lanes micro-batches in flight.

M = N x lanes micro-batches; each tick a stage runs one group of ``lanes`` micro-batches
concurrently on that many HIP streams.  Timed region = ticks [t_a, t_b) with the pipeline full:
t_a = (M + W*M)/L + (P-1), t_b = t_a + K*M/L, i.e. exactly K decode steps of every sequence,
bracketed on every rank by device-synchronize + barrier; the reported time is the max over ranks.
p50 per-token latency = median interval between consecutive tokens of one sequence (M/L ticks),
from device events on the last stage (host timestamps on CPU).

Failure handling: the process group carries a timeout (``EDGELLM_PG_TIMEOUT_S``),
and a heartbeat ``Watchdog`` (``EDGELLM_WATCHDOG_S``, default 300 s) aborts a rank that makes no
progress, naming its last tick, so torchrun tears the job down instead of hanging.
Every rank reports its per-tick compute, P2P wait and bubble fraction over the timed window
(``per_rank`` in the result).  Runs on CPU with gloo when no GPU is present (``--device cpu``),
which is how the multi-process path is tested without GPUs.
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

from ..engine.generate import SamplingParams
from .partition import partition_model, partition_units, stage_costs, unit_stage_costs
from .pipeline import PipelineStage, init_distributed
from .watchdog import Watchdog

_STAT_KEYS = ("compute_ms_per_tick", "p2p_wait_ms_per_tick", "bubble_frac", "p2p_bytes_per_tick", "span_ms",
              "ttft_ms", "host_issue_us_per_tick", "host_post_us_per_tick", "host_finish_us_per_tick",
              "host_compute_us_per_tick")


def _abort_rank(msg: str):
    sys.stderr.write(f"[edgellm watchdog] rank {os.environ.get('RANK', '?')}: {msg}\n")
    sys.stderr.flush()
    os._exit(124)


def run_pipeline_bench(args, build, model_config, kv_dtype=None):
    """``build(args, device, first, last) -> (cfg, stage_model)``; ``model_config(args) -> cfg``;
    ``kv_dtype(args, cfg) -> "bf16" | "int8"`` picks the KV-cache dtype (bf16 when absent)."""
    use_cuda = (args.device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda")
    wd = Watchdog(timeout_s=float(os.environ.get("EDGELLM_WATCHDOG_S", "300")), on_timeout=_abort_rank,
                  name="bench_pipeline").start()
    wd.beat("init_process_group")
    rank, world = init_distributed("nccl" if use_cuda else "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if use_cuda and dist.get_backend() != "nccl":
        # rehearsal: gloo ranks sharing one GPU (EDGELLM_DIST_BACKEND=gloo); collectives on host
        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
    cdev = device if dist.get_backend() == "nccl" else torch.device("cpu")
    cfg = model_config(args)
    wbytes = 1.0 if args.quant != "none" else 2.0
    explicit = args.partition if "," in args.partition else None
    # decode-time cost model, LM head + final norm + sampler in decoder-layer units, measured on
    # MI355X at 256 rows (profiles/rocprof_bench_default_r3_kernel_stats.csv: layer ~227 us; bf16
    # head GEMM 82 us + sampler 25 us + norm/embed ~10 us) -> 0.52; int8 head ~0.35 (estimate,
    # parallel/partition.py::layer_costs); bf16 models 0.4
    hcl = (0.35 if getattr(args, "lm_head", "bf16") == "int8" else 0.52) if args.quant != "none" else 0.4
    L = max(1, getattr(args, "lanes", 1))
    slack = max(0, int(getattr(args, "pp_slack", 0)))
    # LM head split by vocabulary over the ranks (bf16 head; the bench's sampling shards)
    vs = (world > 1 and getattr(args, "pp_vocab_split", "off") == "on" and getattr(args, "lm_head", "bf16") != "int8")
    # micro-batch groups in flight: P (one per stage), or D (P - 1) + 2 with D = 1 + slack ticks per hop;
    # the vocab split D (P + 1) (the token reaches rank 0 two hops later)
    if vs:
        n_groups = (1 + slack) * (world + 1)
    else:
        n_groups = world if slack == 0 or world == 1 else (1 + slack) * (world - 1) + 2
    M, P, b, T = n_groups * L, world, args.micro_batch, args.prompt_len
    kvb = 1.0 if kv_dtype is not None and kv_dtype(args, cfg) == "int8" else 2.0
    unit_kw = dict(rows=b, ctx=T + args.warmup + (args.steps + 1) // 2, weight_bytes=wbytes, kv_bytes=kvb,
                   head_bytes=1.0 if getattr(args, "lm_head", "bf16") == "int8" else 2.0)
    if args.partition == "units" and not explicit:
        ubounds = partition_units(cfg, world, head_split=vs, **unit_kw)
    else:
        bounds = partition_model(cfg, world, "uniform" if args.partition == "uniform" else "balanced",
                                 weight_bytes=wbytes, explicit=explicit, head_cost_layers=hcl)
        ubounds = [2 * x for x in bounds]
    ucost = unit_stage_costs(cfg, ubounds, head_split=vs, **unit_kw)
    wd.beat("build")
    _, model = build(args, device, units=(ubounds[rank], ubounds[rank + 1]))
    shard = None
    if vs:
        from .vocab_head import build_head_shard
        shard = build_head_shard(cfg, rank, world, model=model, seed=args.seed, dtype=torch.bfloat16, device=device,
                                 checkpoint=getattr(args, "checkpoint", None))
    W, K = args.warmup, args.steps
    S = W + K + 1
    g = torch.Generator().manual_seed(args.seed)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)] if rank == 0 else None
    wd.beat("stage init (communicator warm-up)")
    # the stage's constructor joins every rank in one collective (eager RCCL communicator)
    stage = PipelineStage(model, rank, world, b, M, max_seq=T + S + 8, use_graphs=not args.no_graphs,
                          headinfer_heads=getattr(args, "headinfer_heads", None), lanes=L,
                          kv_dtype=kv_dtype(args, cfg) if kv_dtype is not None else "bf16", slack=slack,
                          vocab_split=vs, head_shard=shard)
    if use_cuda:
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(device)
    # ticks count item groups of L micro-batches (one per lane); the last stage lags D (P - 1)
    D = 1 + slack
    t_a = (M + W * M) // L + D * (P - 1)
    t_b = t_a + K * M // L
    # prefill window: tick 0 to the first tick after every prefill group left the last stage
    # (synchronised like the timed window; it ends before the warm-up decodes are timed)
    t_p = M // L + D * (P + 1 if vs else P - 1)
    marks = {}
    stamps = []

    def hook(t):
        if t in (0, t_p, t_a, t_b):
            if use_cuda:
                torch.cuda.synchronize()
            dist.barrier()
            if use_cuda:
                torch.cuda.synchronize()
            marks[t] = time.perf_counter()
        if stage.is_last and t_a <= t <= t_b and (t - t_a) % (M // L) == 0:
            if use_cuda:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                stamps.append(ev)
            else:
                stamps.append(time.perf_counter())

    sp = SamplingParams(max_new_tokens=S + 1, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)
    fault = None
    if os.environ.get("EDGELLM_FAULT_KILL_RANK", "") == str(rank):
        # fault injection (tests): this rank dies hard at its first tick, as a crashed GPU process would
        def fault(t):
            sys.stderr.write(f"[edgellm fault] rank {rank} killed at tick {t}\n")
            sys.stderr.flush()
            os._exit(137)
    dist.barrier()
    res_stage = stage.run(prompts, T, sp, S, seed=args.seed, hook=hook, watchdog=wd, stats_window=(t_a, t_b),
                          fault=fault)
    wd.beat("report")
    fdt = torch.float64
    dt = torch.tensor([marks[t_b] - marks[t_a], marks[t_p] - marks[0]], device=cdev, dtype=fdt)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    lat = torch.zeros(1, device=cdev, dtype=fdt)
    if stage.is_last and len(stamps) > 1:
        if use_cuda:
            iv = sorted(stamps[i - 1].elapsed_time(stamps[i]) for i in range(1, len(stamps)))
        else:
            iv = sorted((stamps[i] - stamps[i - 1]) * 1e3 for i in range(1, len(stamps)))
        lat[0] = iv[len(iv) // 2]
    dist.all_reduce(lat, op=dist.ReduceOp.MAX)
    mem = torch.tensor([torch.cuda.max_memory_allocated(device) / 1e9 if use_cuda else 0.0], device=cdev, dtype=fdt)
    dist.all_reduce(mem, op=dist.ReduceOp.MAX)
    # per-rank window statistics, gathered to every rank as one [world, k] tensor
    mine = torch.tensor([[float(res_stage.stats.get(k, float("nan"))) for k in _STAT_KEYS]], device=cdev, dtype=fdt)
    allst = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allst, mine)
    elapsed, prefill_s = float(dt[0].item()), float(dt[1].item())
    res = None
    if rank == 0:
        tokens = K * M * b
        per_rank = []
        for r, row in enumerate(allst):
            d = {k: round(float(v), 4) for k, v in zip(_STAT_KEYS, row[0].tolist()) if v == v}
            d.update(rank=r, units=[ubounds[r], ubounds[r + 1]], layers=[ubounds[r] / 2, ubounds[r + 1] / 2])
            per_rank.append(d)
        ttft = [d["ttft_ms"] for d in per_rank if "ttft_ms" in d]
        res = dict(value=tokens / elapsed, ms_per_step=elapsed / K * 1e3, p50=float(lat.item()), global_batch=M * b,
                   prefill_tps=M * b * T / prefill_s if prefill_s > 0 else 0.0,
                   mem_gb=float(mem.item()), partition=[u / 2 for u in ubounds], world_size=world, per_rank=per_rank,
                   stage_cost_model_us=[round(c, 1) for c in ucost],
                   stage_cost_spread=round(max(ucost) / (sum(ucost) / len(ucost)), 4), slack=slack,
                   micro_batches_in_flight=M, vocab_split=vs,
                   bubble_frac_max=max(d.get("bubble_frac", 0.0) for d in per_rank),
                   host_issue_us_per_tick_max=max((d.get("host_issue_us_per_tick", 0.0) for d in per_rank),
                                                  default=0.0),
                   ttft_ms=ttft[0] if ttft else None,
                   # HIP streams per rank against the box's hardware queues (GPU_MAX_HW_QUEUES, 4 by
                   # default): one compute stream per lane, one RCCL-internal stream per communicator
                   streams=dict(compute=L, comm_groups=len({id(g) for g in stage.lane_groups}),
                                hw_queues=int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))))
    dist.barrier()
    wd.stop()
    dist.destroy_process_group()
    return res

"""Multi-GPU leg of bench.py: pipeline of N stages (one per GPU), N micro-batches in flight.

M = N x lanes micro-batches; each tick a stage runs one group of ``lanes`` micro-batches
concurrently on that many HIP streams.  Timed region = ticks [t_a, t_b) with the pipeline full:
t_a = (M + W*M)/L + (P-1), t_b = t_a + K*M/L, i.e. exactly K decode steps of every sequence,
bracketed on every rank by device-synchronize + barrier; the reported time is the max over ranks.
p50 per-token latency = median interval between consecutive tokens of one sequence (M/L ticks),
from device events on the last stage (host timestamps on CPU).
Runs on CPU with gloo when no GPU is present (``--device cpu``), which is how the multi-process
path is tested without GPUs.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from ..engine.generate import SamplingParams
from .partition import partition_model, stage_costs
from .pipeline import PipelineStage, init_distributed


def run_pipeline_bench(args, build, model_config):
    """``build(args, device, first, last) -> (cfg, stage_model)``; ``model_config(args) -> cfg``."""
    use_cuda = (args.device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda")
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
    # decode-time cost model: LM head + sampler ~0.6 of a W8A8 decoder layer (0.4 of a bf16 one),
    # measured on MI355X at 64 rows per lane (parallel/partition.py::layer_costs)
    hcl = 0.6 if args.quant != "none" else 0.4
    bounds = partition_model(cfg, world, "uniform" if args.partition == "uniform" else "balanced",
                             weight_bytes=wbytes, explicit=explicit, head_cost_layers=hcl)
    _, model = build(args, device, first=bounds[rank], last=bounds[rank + 1])
    L = max(1, getattr(args, "lanes", 1))
    M, P, b, T = world * L, world, args.micro_batch, args.prompt_len
    W, K = args.warmup, args.steps
    S = W + K + 1
    g = torch.Generator().manual_seed(args.seed)
    prompts = [torch.randint(0, cfg.vocab_size, (b, T), generator=g) for _ in range(M)] if rank == 0 else None
    stage = PipelineStage(model, rank, world, b, M, max_seq=T + S + 8, use_graphs=not args.no_graphs,
                          headinfer_heads=getattr(args, "headinfer_heads", None), lanes=L)
    # initialise the communicator with a collective every rank joins
    x = torch.ones(1, device=cdev)
    dist.all_reduce(x)
    if use_cuda:
        torch.cuda.synchronize()
    # ticks count item groups of L micro-batches (one per lane)
    t_a = (M + W * M) // L + (P - 1)
    t_b = t_a + K * M // L
    marks = {}
    stamps = []

    def hook(t):
        if t in (t_a, t_b):
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
    stage.run(prompts, T, sp, S, seed=args.seed, hook=hook)
    fdt = torch.float64
    dt = torch.tensor([marks[t_b] - marks[t_a]], device=cdev, dtype=fdt)
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
    elapsed = float(dt.item())
    res = None
    if rank == 0:
        tokens = K * M * b
        res = dict(value=tokens / elapsed, ms_per_step=elapsed / K * 1e3, p50=float(lat.item()), global_batch=M * b,
                   mem_gb=float(mem.item()), partition=bounds,
                   stage_cost_mb=[round(c / 1e6, 1) for c in stage_costs(cfg, bounds, wbytes, head_cost_layers=hcl)])
    dist.barrier()
    dist.destroy_process_group()
    return res

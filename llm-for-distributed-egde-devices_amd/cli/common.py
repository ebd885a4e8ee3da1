"""Shared CLI plumbing: device selection, argument groups beyond the reference's flags."""
from __future__ import annotations

import argparse
from typing import List

import torch


def add_runtime_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    g = p.add_argument_group("edgellm runtime (not in the reference)")
    g.add_argument("--quant", default=None, choices=["none", "w8a8_smoothquant", "w8a8", "llm_int8", "cpu_dynamic"],
                   help="quantisation mode (default: none, or from YAML quant.mode)")
    g.add_argument("--precision", default=None, help="fp16|bf16|fp32 (GPU: fp16 and bf16 kernels; fp32 and INT8 models run bf16)")
    g.add_argument("--devices", default=None, help="comma list, e.g. cuda:0,cuda:1 (agents round-robin)")
    g.add_argument("--num_samples", type=int, default=None, help="evaluate only the first N samples")
    g.add_argument("--seed", type=int, default=0, help="sampling seed (the reference sets none)")
    g.add_argument("--max_seq", type=int, default=2048, help="KV-cache capacity per sequence")
    g.add_argument("--progress", default=None, help="JSONL progress file (resume after a crash)")
    g.add_argument("--base_model_path", default=None, help="directory holding downloaded checkpoints")
    g.add_argument("--no_legacy_decode", action="store_true",
                   help="score only generated text (the reference decodes prompt + answer)")
    g.add_argument("--no_reference_in_refiner", action="store_true",
                   help="do not leak the gold answer into the refiner prompt")
    g.add_argument("--merge", default=None, choices=["refine", "vote"], help="ensemble merge (default refine)")
    g.add_argument("--serial", action="store_true", help="run agents one after another (reference behaviour)")
    g.add_argument("--headinfer_heads", type=int, default=None,
                   help="HeadInfer: KV heads per layer resident on the GPU, the rest in pinned host memory "
                        "(default: YAML offload.gpu_kv_budget_heads when offload.headinfer is true)")
    g.add_argument("--prefill_chunk", type=int, default=None, help="chunked prefill size (YAML offload.chunk_size)")
    g.add_argument("--pp_size", type=int, default=None,
                   help="split each model's layers over this many GPUs (YAML parallel.pp_size; agents[].gpus wins)")
    g.add_argument("--batch_size", type=int, default=None,
                   help="questions decoded together per agent (YAML parallel.microbatches; 1 = the reference)")
    g.add_argument("--kv_dtype", default=None, choices=["bf16", "int8"], help="KV-cache dtype (default bf16)")
    g.add_argument("--partition", default=None,
                   help="torchrun pipelines: balanced | units (half-layer stage bounds from the decode cost model) | "
                        "uniform | '8,8,8,8' (YAML parallel.partition)")
    g.add_argument("--pp_lanes", type=int, default=None,
                   help="torchrun pipelines: micro-batches each stage runs concurrently (YAML parallel.lanes)")
    g.add_argument("--pp_slack", type=int, default=None,
                   help="torchrun pipelines: extra ticks per hop, P2P overlapped with compute (YAML parallel.slack)")
    g.add_argument("--pp_vocab_split", default=None, choices=["on", "off"],
                   help="torchrun pipelines: split the LM head by vocabulary over the stages, rank 0 merging "
                        "the sampler's candidates (default on; YAML parallel.vocab_split)")
    g.add_argument("--calib", default=None, choices=["stage", "full"],
                   help="torchrun + w8a8_smoothquant: calibrate each stage on the activations it receives "
                        "(stage, default) or the full model on every rank (full) (YAML parallel.calib)")
    g.add_argument("--metrics_jsonl", default=None, help="append structured per-sample metrics here")
    return p


def pick_devices(spec: str = None) -> List[torch.device]:
    if spec:
        return [torch.device(s.strip()) for s in spec.split(",") if s.strip()]
    if torch.cuda.is_available():
        return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    return [torch.device("cpu")]


def pop_runtime(args: argparse.Namespace) -> dict:
    """Remove runtime-only keys so the remaining namespace is the reference's flag set."""
    keys = ["quant", "precision", "devices", "num_samples", "seed", "max_seq", "progress", "base_model_path",
            "no_legacy_decode", "no_reference_in_refiner", "merge", "serial", "headinfer_heads", "metrics_jsonl",
            "prefill_chunk", "pp_size", "batch_size", "kv_dtype", "partition", "pp_lanes", "pp_slack", "calib",
            "pp_vocab_split"]
    return {k: args.__dict__.pop(k) for k in keys if k in args.__dict__}


def resolve_runtime(cfg, rt: dict) -> dict:
    """Fold the YAML sections the CLIs act on (``parallel``, ``offload``) into the runtime dict;
    an explicit flag wins.  Returns rt with: pp_size, batch_size, headinfer_heads, prefill_chunk."""
    rt = dict(rt)
    if rt.get("pp_size") is None:
        rt["pp_size"] = max(1, int(cfg.parallel.pp_size or 1))
    if rt.get("batch_size") is None:
        rt["batch_size"] = max(1, int(cfg.parallel.microbatches or 1))
    if rt.get("headinfer_heads") is None and cfg.offload.headinfer:
        rt["headinfer_heads"] = cfg.offload.gpu_kv_budget_heads if cfg.offload.gpu_kv_budget_heads is not None else 0
    if rt.get("prefill_chunk") is None:
        rt["prefill_chunk"] = cfg.offload.chunk_size
    par = cfg.parallel
    rt["partition"] = rt.get("partition") or getattr(par, "partition", "balanced") or "balanced"
    rt["pp_lanes"] = max(1, int(rt.get("pp_lanes") or getattr(par, "lanes", 1) or 1))
    rt["pp_slack"] = max(0, int(rt.get("pp_slack") if rt.get("pp_slack") is not None else getattr(par, "slack", 0) or 0))
    rt["calib"] = rt.get("calib") or getattr(par, "calib", "stage") or "stage"
    vs = rt.get("pp_vocab_split")
    rt["pp_vocab_split"] = (vs == "on") if vs is not None else bool(getattr(par, "vocab_split", True))
    rt.setdefault("kv_dtype", None)
    rt["kv_dtype"] = rt["kv_dtype"] or "bf16"
    return rt


def build_generator(model, rt: dict, max_batch: int = 1):
    """The decode engine for one agent / model as the runtime options ask: HeadInfer KV offload
    (``headinfer_heads``, chunked prefill), int8 KV cache, or the resident bf16 cache."""
    from ..engine import Generator
    from ..engine.kv_cache import resolve_kv_dtype
    max_seq = rt.get("max_seq", 2048)
    h_on = rt.get("headinfer_heads")
    if h_on is not None and h_on < model.cfg.num_kv_heads:
        assert not hasattr(model, "make_kv"), "HeadInfer offload runs on a single-device model"
        from ..offload import HeadInferKV
        chunk = min(int(rt.get("prefill_chunk") or 4096), max_seq)
        kv = HeadInferKV(model.cfg, max_batch, max_seq, int(h_on), model.device, chunk_size=chunk, dtype=model.dtype)
        return Generator(model, max_batch=max_batch, max_seq=max_seq, kv=kv)
    kvd = resolve_kv_dtype(rt.get("kv_dtype") or "bf16", model.cfg, model.dtype, model.device)
    return Generator(model, max_batch=max_batch, max_seq=max_seq, kv_dtype=kvd,
                     prefill_chunk=rt.get("prefill_chunk") if h_on is not None else None)


def pp_launch(rt: dict):
    """Under ``torchrun`` (WORLD_SIZE > 1) every model runs as a pipeline over the ranks, one
    process per GPU (parallel/pp_engine.py): returns (rank, world, device) after initialising the
    process group (RCCL with a GPU per rank, gloo on CPU); None for a single-process run.
    ``pp_size`` must then equal the world size (or be left unset)."""
    from ..parallel.pp_engine import distributed_world
    world = distributed_world()
    if world <= 1:
        return None
    import os
    from ..parallel.pipeline import init_distributed
    pp = int(rt.get("pp_size") or 1)
    assert pp in (1, world), f"--pp_size {pp} under a {world}-rank torchrun launch"
    want_cpu = (rt.get("devices") or "").startswith("cpu") or not torch.cuda.is_available()
    rank, world = init_distributed("gloo" if want_cpu else "nccl")
    import atexit
    import torch.distributed as dist
    # tear the process group down before interpreter exit (a live group's threads abort the
    # process at exit, which torchrun reports as a failed rank)
    atexit.register(lambda: dist.is_initialized() and dist.destroy_process_group())
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not want_cpu and dist.get_backend() != "nccl":
        # rehearsal (EDGELLM_DIST_BACKEND=gloo): more ranks than GPUs share them, P2P host-staged
        local %= max(1, torch.cuda.device_count())
    dev = torch.device("cpu") if want_cpu else torch.device("cuda", local)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    return rank, world, dev


def agent_group(ranks, world: int):
    """Process group of an agent's ranks: the default group when it spans the world, else a new
    group.  Every rank must call this for every agent in the same order (dist.new_group)."""
    import torch.distributed as dist
    if list(ranks) == list(range(world)):
        return None
    return dist.new_group(list(ranks))


def build_pp_engine(model_id: str, precision: str, quant: str, rt: dict, launch, tag: int, max_batch: int = 1,
                    gpus=None):
    """This rank's stage of ``model_id`` behind a ``PipelineGenerator`` (the Generator interface
    on the driver, rank 0).  ``gpus`` (YAML ``agents[].gpus``): the agent's rank group — one
    process per GPU, so GPU index = rank; default all ranks.  A rank outside the group holds a
    stub engine.  Returns (engine, tokenizer, source, bounds)."""
    from ..engine.kv_cache import resolve_kv_dtype
    from ..parallel.pp_engine import PipelineGenerator, _cfg_of, load_stage
    rank, world, dev = launch
    ranks = sorted(int(g) for g in gpus) if gpus else list(range(world))
    assert ranks and all(0 <= r < world for r in ranks) and len(set(ranks)) == len(ranks), \
        f"agent gpus {gpus} must be distinct ranks of the {world}-rank launch"
    group = agent_group(ranks, world)
    kvd = rt.get("kv_dtype") or "bf16"
    lanes, slack = int(rt.get("pp_lanes") or 1), int(rt.get("pp_slack") or 0)
    vs = bool(rt.get("pp_vocab_split", False)) and len(ranks) > 1
    common = dict(max_batch=max_batch, max_seq=rt.get("max_seq", 2048), tag=tag, group=group, ranks=ranks,
                  lanes=lanes, slack=slack, vocab_split=vs)
    if rank not in ranks:
        cfg, tok, source = _cfg_of(model_id, precision, torch.device("cpu"), rt.get("base_model_path"))
        eng = PipelineGenerator(None, -1, len(ranks), cfg=cfg, device=dev, **common)
        return eng, tok, source, None
    s_idx = ranks.index(rank)
    M, b = PipelineGenerator.geometry(len(ranks), max_batch, lanes, slack, vocab_split=vs)
    stage, tok, source, bounds = load_stage(model_id, precision, quant, dev, rt.get("base_model_path"), s_idx,
                                            len(ranks), partition=rt.get("partition") or "balanced", group=group,
                                            ranks=ranks, calib=rt.get("calib") or "stage", rows=b,
                                            ctx=min(int(rt.get("max_seq", 2048)), 256))
    kvd = resolve_kv_dtype(kvd, stage.cfg, stage.dtype, dev)
    shard = None
    if vs:
        # every member gets its rows of the head from the last stage (one P2P per rank, at load)
        from ..parallel.vocab_head import shard_from_last_stage
        shard = shard_from_last_stage(stage, stage.cfg, s_idx, len(ranks), group=group, ranks=ranks, device=dev)
    eng = PipelineGenerator(stage, s_idx, len(ranks), kv_dtype=kvd, head_shard=shard, **common)
    return eng, tok, source, bounds

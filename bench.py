#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): whole-node decode tokens/sec + p50 per-token latency,
Llama-2-7B, SmoothQuant W8A8 INT8, layer-split across N GPUs of one node.

    python bench.py --gpus 1 --steps 64 --warmup 8
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 64 --warmup 8

Work per step: every in-flight sequence decodes one token, sampled with the reference's config
(T=0.7, top-k 50, top-p 0.9, repetition penalty 1.1 — Code/others/config.yaml:3-7).
N = 1 runs graph-captured Generators on one GPU; N > 1 runs the RCCL pipeline with one stage
(~32/N decoder layers) per GPU and N x lanes micro-batches in flight.  Every GPU decodes ``lanes``
micro-batches concurrently on separate HIP streams (default 2 x 256 sequences: each micro-batch's
decode GEMMs read a weight once for its 256 rows, and one lane's HBM-bound attention overlaps the
other lane's GEMMs), so per-GPU work per step is constant (weak scaling: global batch =
micro-batch x lanes x N).
Weights: random-init Llama-2-7B architecture (seeded by global parameter name, so a stage's
bf16 weights equal the unsplit model's), SmoothQuant-calibrated on synthetic tokens: at N = 1
the full model; at N > 1 each rank builds only its stage and calibrates it on the activations
the previous stage sends (``--calib stage``, default; ``--calib full`` builds + calibrates the
full model on every rank and cuts the stage, bit-identical INT8 weights for every split).
Data: random prompt ids.  ``--device cpu --model tiny:llama``
exercises the same code paths on CPU (gloo) for tests.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm.engine import Generator, SamplingParams  # noqa: E402
from edgellm.engine.generate import LaneGenerator  # noqa: E402
from edgellm.models import build_model, get_config, tiny  # noqa: E402
from edgellm.quant import quantize_head, quantize_model, synthetic_calibration  # noqa: E402
from edgellm.quant.smoothquant import smoothquant_stage  # noqa: E402
from edgellm.utils.tracing import MetricsWriter, trace_range  # noqa: E402

METRIC = "tokens/sec (whole node) + p50 per-token latency, Llama-2-7B INT8 split 1/2/4/8"
# no published value for this metric; the closest published point is the reference's
# single-stream INT8 decode rate (Llama-3.2-1B, bitsandbytes LLM.int8, A100): 25.8326 tok/s.
BASELINE_TPS = 25.8326


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="llama-2-7b")
    ap.add_argument("--quant", default="w8a8_smoothquant", choices=["none", "w8a8_smoothquant", "w8a8"])
    ap.add_argument("--checkpoint", default=None,
                    help="an edgellm INT8 checkpoint directory (python -m edgellm.cli.quantize): every rank reads "
                         "only its stage instead of building + calibrating the full bf16 model")
    ap.add_argument("--micro-batch", type=int, default=256,
                    help="sequences per micro-batch (256: the largest the fused decode GEMMs take — the 129-256-row "
                         "kernels stream every weight once for all 256 sequences; 16-128 trade tok/s for latency)")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--lanes", type=int, default=2,
                    help="micro-batches each GPU decodes concurrently on separate HIP streams (own graphs/pools): "
                         "one lane's HBM-bound attention runs beside the other's ingest-bound GEMMs (2 x 256: "
                         "41.9k tok/s at p50 12.2 ms; 1 x 256: 35.8k at 7.1 ms)")
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "int8"],
                    help="KV cache: bf16 (default) or int8 with per-(token, head) scales (half the KV bytes: 1.6x faster attention at >= 512 keys, neutral at the 128-token bench context)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--lm-head", default="bf16", choices=["bf16", "int8"],
                    help="int8: W8A8 LM head (per-channel weights, per-token activations); default bf16 "
                         "like the reference")
    ap.add_argument("--force-pipeline", action="store_true",
                    help="N = 1: time the RCCL PipelineStage engine (world-1 process group, device bound) "
                         "instead of the Generator, same config")
    ap.add_argument("--device", default=None, help="cuda (default when available) | cpu (gloo, tests)")
    ap.add_argument("--partition", default="units",
                    help="units (balanced over half-layer units: a stage boundary may fall between a layer's "
                         "attention and MLP halves) | balanced (whole layers) | uniform | explicit '9,8,8,7'")
    ap.add_argument("--calib", default="stage", choices=["stage", "full"],
                    help="N > 1: SmoothQuant calibration per stage over P2P (each rank builds only its stage) "
                         "or of the full model on every rank")
    ap.add_argument("--pp-slack", type=int, default=0,
                    help="N > 1: extra ticks per stage hop (1 = 2N micro-batches in flight, every RCCL hop "
                         "overlapped with a tick of compute; doubles the per-token latency)")
    ap.add_argument("--pp-vocab-split", default="on", choices=["on", "off"],
                    help="N > 1: split the LM head by vocabulary over every rank (each rank its logits slice + "
                         "sampler phase 1, rank 0 the merge) instead of the whole head on the last stage; one "
                         "more micro-batch group in flight (parallel/vocab_head.py)")
    ap.add_argument("--latency-point", default="auto", choices=["auto", "off", "int8", "both"],
                    help="also report batch-1 p50 per-token latency (single GPU): int8 = the benchmark model at "
                         "micro-batch 1, both = plus a bf16 copy of the model (13.5 GB more, built for this only); "
                         "auto = int8 on a GPU, off on CPU")
    ap.add_argument("--prefill-chunk", type=int, default=None,
                    help="chunked prefill size with HeadInfer (default: the whole prompt in one chunk)")
    ap.add_argument("--headinfer-heads", type=int, default=None,
                    help="HeadInfer: KV heads per layer kept on the GPU, the rest offloaded to pinned host memory")
    ap.add_argument("--metrics-out", default=os.environ.get("EDGELLM_METRICS"),
                    help="append the result record (plus HBM peak) to this JSONL file")
    return ap.parse_args(argv)


def model_config(args):
    if getattr(args, "checkpoint", None):
        from edgellm.quant.checkpoint import checkpoint_config
        cfg = checkpoint_config(args.checkpoint)
    elif args.model.startswith("tiny:"):
        cfg = tiny(args.model.split(":", 1)[1], num_layers=8)   # 8 layers: splits up to 8 stages
    else:
        cfg = get_config(args.model)
    need = args.prompt_len + args.warmup + args.steps + 16
    if need > cfg.max_position_embeddings:      # long-context runs (HeadInfer): extend the RoPE table
        cfg = cfg.replace(max_position_embeddings=need)
    return cfg


def build(args, device, first=0, last=None, units=None):
    """Stage [first, last) of the benchmark model (or the half-layer units ``units=(ua, ub)`` of a
    sub-layer split), quantised exactly as the unsplit model."""
    cfg = model_config(args)
    dtype = torch.bfloat16
    if getattr(args, "checkpoint", None):
        # an edgellm INT8 checkpoint (python -m edgellm.cli.quantize): this stage's tensors only
        from edgellm.quant.checkpoint import load_quantized
        model = load_quantized(args.checkpoint, device=device, first=first, last=last, dtype=dtype, units=units)
        if getattr(args, "lm_head", "bf16") == "int8" and model.has_head:
            model = quantize_head(model)
        if device.type == "cuda":
            torch.cuda.empty_cache()
            torch.cuda.synchronize()
        return cfg, model
    if args.quant == "w8a8_smoothquant" and getattr(args, "calib", "stage") == "stage" and _pipeline_rank() is not None:
        # per-stage SmoothQuant: this rank builds only its stage and calibrates it on the bf16
        # activations the previous stage sends over the pipeline's P2P path (no full model here)
        import torch.distributed as dist
        from edgellm.quant.smoothquant import smoothquant_stage_p2p
        rank, world = _pipeline_rank()
        calib = synthetic_calibration(cfg, n=2, T=64, device=device, seed=args.seed)
        cdev = device if dist.get_backend() == "nccl" else torch.device("cpu")

        def recv_prev(shape, dt):
            t = torch.empty(shape, dtype=dt, device=cdev)
            dist.recv(t, rank - 1)
            return t

        model = smoothquant_stage_p2p(cfg, calib, recv_prev, lambda t: dist.send(t.to(cdev), rank + 1),
                                      first=first, last=last, units=units, dtype=dtype, device=device,
                                      seed=args.seed)
    elif args.quant == "w8a8_smoothquant":
        full = build_model(cfg, dtype=dtype, device=device, seed=args.seed)
        calib = synthetic_calibration(cfg, n=2, T=64, device=device, seed=args.seed)
        model = smoothquant_stage(full, first, cfg.num_layers if last is None else last, calib, device=device,
                                  units=units)
        del full
    else:
        model = build_model(cfg, dtype=dtype, device=device, first=first, last=last, seed=args.seed, units=units)
        if args.quant != "none":
            model = quantize_model(model, args.quant)
    if getattr(args, "lm_head", "bf16") == "int8" and model.has_head:
        model = quantize_head(model)
    if device.type == "cuda":
        torch.cuda.empty_cache()
        torch.cuda.synchronize()
    return cfg, model


def _pipeline_rank():
    """(rank, world) inside a multi-rank pipeline launch with the process group up, else None."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_rank(), dist.get_world_size()
    return None


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize()


def run_single(args):
    device = torch.device(args.device or ("cuda:0" if torch.cuda.is_available() else "cpu"))
    if device.type == "cuda":
        torch.cuda.set_device(device)
    t_build = time.perf_counter()
    cfg, model = build(args, device)
    t_build = time.perf_counter() - t_build
    if device.type == "cuda":
        torch.cuda.reset_peak_memory_stats(device)   # report the serving peak, not the build's
    B = args.micro_batch
    total_new = args.warmup + args.steps + 2
    max_seq = args.prompt_len + total_new + 8
    kv = None
    if args.headinfer_heads is not None and args.headinfer_heads < cfg.num_kv_heads:
        from edgellm.offload import HeadInferKV
        kv = HeadInferKV(cfg, B, max_seq, args.headinfer_heads, device,
                         chunk_size=max(1, min(args.prompt_len, args.prefill_chunk or args.prompt_len)),
                         kv_dtype=kv_dtype(args, cfg))
    L = max(1, args.lanes)
    if L > 1:
        assert kv is None, "HeadInfer offload runs one lane"
        gen = LaneGenerator(model, lanes=L, max_batch=B, max_seq=max_seq, use_graphs=not args.no_graphs,
                            kv_dtype=kv_dtype(args, cfg))
    else:
        gen = Generator(model, max_batch=B, max_seq=max_seq, use_graphs=not args.no_graphs, kv=kv,
                        kv_dtype=kv_dtype(args, cfg))
    g = torch.Generator().manual_seed(args.seed)
    prompts = torch.randint(0, cfg.vocab_size, (B * L, args.prompt_len), generator=g).tolist()
    sp = SamplingParams(max_new_tokens=total_new, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)
    gen.start(prompts, sp, seed=args.seed)
    prefill_s = gen._t_prefill if L > 1 else gen._run["t_prefill"]
    ttft_ms = (gen.lanes[0] if L > 1 else gen)._run["t_prefill"] * 1e3   # prefill + first sampled token, lane 0
    gen.step(args.warmup, record_latency=False)
    gen.precapture(args.steps + 1)
    _sync(device)
    lanes = gen.lanes if L > 1 else [gen]
    n_ev = [len(x._run["events"]) for x in lanes]
    t0 = time.perf_counter()
    with trace_range("bench.timed"):
        gen.step(args.steps, record_latency=device.type == "cuda")
        _sync(device)
    dt = time.perf_counter() - t0
    lat = []
    for x, n0 in zip(lanes, n_ev):
        ev = x._run["events"][n0:]
        lat += [ev[i - 1].elapsed_time(ev[i]) for i in range(1, len(ev))]
    lat.sort()
    p50 = lat[len(lat) // 2] if lat else dt / args.steps * 1e3
    p90 = lat[int(len(lat) * 0.9)] if lat else p50
    lmax = lat[-1] if lat else p50
    tokens = B * L * args.steps
    mem = torch.cuda.max_memory_allocated() / 1e9 if device.type == "cuda" else 0.0
    kv_gpu = (kv.gpu_bytes() if kv is not None else gen_kv_bytes(gen)) / 1e9
    graphs = lanes[0]._run["graphs_ok"]
    del gen, lanes
    if device.type == "cuda":
        torch.cuda.empty_cache()
    lat_pts = latency_points(args, device, model, cfg) if args.headinfer_heads is None else {}
    one_lane = {}
    if L > 1 and device.type == "cuda" and args.latency_point != "off":
        # the same micro-batch in ONE lane: the latency side of the lanes trade-off
        one_lane = dict(micro_batch=B, lanes=1, steps=min(args.steps, 20),
                        **batch1_p50(model, cfg, args, device, min(args.steps, 20), rows=B))
        torch.cuda.empty_cache()
    offload = {}
    if kv is not None:
        offload = dict(h_on=kv.h_on, h_off=kv.h_off, chunk_size=kv.chunk_size, h2d_gb=round(kv.bytes_h2d / 1e9, 3),
                       d2h_gb=round(kv.bytes_d2h / 1e9, 3), transports=dict(kv.transports))
    return dict(latency_point=lat_pts, one_lane_point=one_lane, offload=offload, value=tokens / dt, ms_per_step=dt / args.steps * 1e3, p50=p50, p90=p90, lat_max=lmax, global_batch=B * L,
                prefill_tps=B * L * args.prompt_len / prefill_s, build_s=t_build, graphs=graphs,
                mem_gb=mem, partition=[0, cfg.num_layers], ttft_ms=ttft_ms, world_size=1, kv_gpu_gb=kv_gpu,
                kv_host_gb=(kv.host_bytes() / 1e9 if kv is not None else 0.0))


def kv_dtype(args, cfg) -> str:
    """The requested KV-cache dtype where the model supports it (int8 needs head_dim 64 / 128 /
    256; with HeadInfer it applies to every tier: resident, host pool and staging)."""
    if args.kv_dtype == "int8" and cfg.head_dim in (64, 128, 256):
        return "int8"
    return "bf16"


@torch.no_grad()
def batch1_p50(model, cfg, args, device, steps: int, rows: int = 1) -> dict:
    """Decode latency of ``model`` at ``rows`` sequences in one lane (graph-captured, same sampling
    config): p50 / p90 of per-token device-event intervals over ``steps`` tokens after a warm-up."""
    W = max(4, args.warmup)
    max_seq = args.prompt_len + W + steps + 16
    gen = Generator(model, max_batch=rows, max_seq=max_seq, use_graphs=not args.no_graphs,
                    kv_dtype=kv_dtype(args, cfg))
    g = torch.Generator().manual_seed(args.seed + 1)
    prompt = torch.randint(0, cfg.vocab_size, (rows, args.prompt_len), generator=g).tolist()
    sp = SamplingParams(max_new_tokens=W + steps + 2, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)
    gen.start(prompt, sp, seed=args.seed)
    gen.step(W, record_latency=False)
    gen.precapture(steps + 1)
    _sync(device)
    n0 = len(gen._run["events"])
    t0 = time.perf_counter()
    gen.step(steps, record_latency=device.type == "cuda")
    _sync(device)
    dt = time.perf_counter() - t0
    ev = gen._run["events"][n0:]
    lat = sorted(ev[i - 1].elapsed_time(ev[i]) for i in range(1, len(ev))) or [dt / steps * 1e3]
    out = dict(p50_ms=round(lat[len(lat) // 2], 4), p90_ms=round(lat[int(len(lat) * 0.9)], 4),
               tokens_per_s=round(rows * steps / dt, 1), ttft_ms=round(gen._run["t_prefill"] * 1e3, 3))
    del gen
    return out


def latency_points(args, device, model, cfg) -> dict:
    mode = args.latency_point
    if mode == "auto":
        mode = "int8" if device.type == "cuda" else "off"
    if mode == "off":
        return {}
    steps = max(32, args.steps)
    pts = {"micro_batch": 1, "prompt_len": args.prompt_len, "steps": steps}
    pts[args.quant if args.quant != "none" else "bf16"] = batch1_p50(model, cfg, args, device, steps)
    if mode == "both" and args.quant != "none":
        import copy
        a2 = copy.copy(args)
        a2.quant = "none"
        _, m16 = build(a2, device)
        pts["bf16"] = batch1_p50(m16, cfg, a2, device, steps)
        del m16
        if device.type == "cuda":
            torch.cuda.empty_cache()
    return pts


def gen_kv_bytes(gen) -> int:
    lanes = gen.lanes if hasattr(gen, "lanes") else [gen]
    return sum(x.kv.nbytes() for x in lanes)


def run_pipeline(args):
    from edgellm.parallel.bench_pipeline import run_pipeline_bench
    return run_pipeline_bench(args, build, model_config, kv_dtype)


def _world1_env():
    """torchrun-style env for a one-rank process group (``--force-pipeline`` at N = 1)."""
    import socket
    if "MASTER_PORT" not in os.environ:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        s.close()
    for k, v in (("RANK", "0"), ("LOCAL_RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1")):
        os.environ.setdefault(k, v)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv) -> int:
    """``python bench.py --gpus N`` without torchrun: start N fresh rank processes of this script
    (one per GPU, torchrun's env contract: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT) and relay rank 0's stdout (the JSON line).  The parent never touches the GPU and
    never execs; it only waits.  Watchdog: once any rank exits non-zero the others get
    ``EDGELLM_LAUNCH_GRACE_S`` (default 30 s) to finish before they are terminated (a rank blocked
    in a collective on a dead peer would otherwise hang), and ``EDGELLM_LAUNCH_TIMEOUT_S`` (default
    0 = none) bounds the whole job.  Exit code: the worst child's (signals as 128 + signo).
    The reference's multi-device mechanism this replaces: Llama_bf16_updated.py:31
    (``device_map="auto"``)."""
    import signal
    import subprocess
    import threading
    port = _free_port()
    grace = float(os.environ.get("EDGELLM_LAUNCH_GRACE_S", "30"))
    limit = float(os.environ.get("EDGELLM_LAUNCH_TIMEOUT_S", "0"))
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", ROLE_RANK=str(r), ROLE_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TORCHELASTIC_RUN_ID="edgellm-bench")
        env.setdefault("OMP_NUM_THREADS", "1")            # torchrun's default for multi-rank jobs
        # rank 0's stdout is relayed line by line (the one JSON line); other ranks print to stderr
        out = subprocess.PIPE if r == 0 else sys.stderr.fileno()
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
                                      stdout=out, text=True if r == 0 else None))

    def relay(stream):
        for line in stream:
            sys.stdout.write(line)
            sys.stdout.flush()

    th = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    th.start()

    def kill_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    def on_signal(signo, _frame):
        kill_all()
        raise SystemExit(128 + signo)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    t0 = time.monotonic()
    t_fail = None
    try:
        while any(p.poll() is None for p in procs):
            now = time.monotonic()
            if t_fail is None and any(p.returncode not in (None, 0) for p in procs):
                t_fail = now
                bad = [(i, p.returncode) for i, p in enumerate(procs) if p.returncode not in (None, 0)]
                sys.stderr.write(f"[bench launcher] rank(s) {bad} failed; terminating the rest in {grace:.0f} s\n")
            if (t_fail is not None and now - t_fail > grace) or (limit > 0 and now - t0 > limit):
                sys.stderr.write("[bench launcher] terminating ranks still running\n")
                kill_all()
                deadline = time.monotonic() + 10
                while any(p.poll() is None for p in procs) and time.monotonic() < deadline:
                    time.sleep(0.1)
                kill_all(signal.SIGKILL)
                if t_fail is None:
                    t_fail = now
            time.sleep(0.1)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    th.join(timeout=5)
    rcs = [p.wait() for p in procs]
    worst = 0
    for rc in rcs:
        code = 128 - rc if rc < 0 else rc
        worst = max(worst, code)
    if limit > 0 and worst == 0 and t_fail is not None:
        worst = 124
    if worst:
        sys.stderr.write(f"[bench launcher] job failed: rank exit codes {rcs}\n")
    return worst


def main(argv=None):
    raw = list(sys.argv[1:] if argv is None else argv)
    args = parse(raw)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun around us: start the N rank processes ourselves (the parent stays GPU-free)
        raise SystemExit(launch_ranks(args.gpus, raw))
    if args.headinfer_heads is not None:
        args.lanes = 1          # the HeadInfer offload is host-orchestrated: one lane per GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.force_pipeline and world == 1 and args.gpus == 1:
        _world1_env()
        world = 1
        res = run_pipeline(args)
    elif args.gpus > 1 or world > 1:
        assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with torchrun"
        res = run_pipeline(args)
    else:
        res = run_single(args)
    if res is None:  # non-zero ranks
        return None
    out = {
        "metric": METRIC,
        "value": round(res["value"], 2),
        "unit": "tokens/s",
        "n_gpus": args.gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(res["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        # no published value exists for this metric (Llama-2-7B INT8 split 1/2/4/8)
        "vs_baseline": None,
        "closest_published": {"what": "single-stream INT8 decode tok/s, Llama-3.2-1B, bitsandbytes LLM.int8, "
                                      "A100 (ACL.pdf p.7 Table 3) - different model size and batch",
                              "value": BASELINE_TPS},
        "dtype": "int8" if args.quant != "none" else "bf16",
        "data": f"synthetic (random-init {args.model} weights"
                + (", SmoothQuant-calibrated on random tokens" if args.quant == "w8a8_smoothquant" else "")
                + "; random prompts)",
        "config": {"model": args.model, "global_batch": res["global_batch"], "seq_len": args.prompt_len,
                   "parallelism": f"pp{args.gpus}", "quant": args.quant, "micro_batch": args.micro_batch,
                   "micro_batches_in_flight": res.get("micro_batches_in_flight", max(1, args.gpus) * max(1, args.lanes)),
                   "lanes": max(1, args.lanes), "partition": res.get("partition"),
                   "sampling": "T=0.7 top_k=50 top_p=0.9 rep=1.1",
                   "headinfer_heads": args.headinfer_heads,
                   "kv_cache": ("int8, one fp32 scale per (token, head)" if kv_dtype(args, model_config(args)) == "int8"
                                else "bf16"),
                   "compute": ("W8A8 INT8 MFMA GEMMs, bf16 norms / softmax, "
                               + ("W8A8 int8 LM head" if args.lm_head == "int8" else "bf16 LM head")
                               + (f" split by vocabulary over {args.gpus} ranks" if res.get("vocab_split") else "")
                               if args.quant != "none" else "bf16 GEMMs / attention / norms")},
        "p50_token_latency_ms": round(res["p50"], 4),
        "p90_token_latency_ms": round(res.get("p90", res["p50"]), 4),
        "max_token_latency_ms": round(res.get("lat_max", res["p50"]), 4),
        "prefill_tokens_per_s": round(res.get("prefill_tps", 0.0), 1),
        "peak_mem_gb": round(res.get("mem_gb", 0.0), 2),
        "world_size": res.get("world_size", args.gpus),
        "engine": "PipelineStage" if (args.force_pipeline or args.gpus > 1) else "Generator",
    }
    if res.get("ttft_ms") is not None:
        out["ttft_ms"] = round(res["ttft_ms"], 3)
    for k in ("kv_gpu_gb", "kv_host_gb"):
        if k in res:
            out[k] = round(res[k], 3)
    if res.get("offload"):
        out["offload"] = res["offload"]
    if res.get("latency_point"):
        out["latency_point"] = res["latency_point"]
    if res.get("one_lane_point"):
        out["one_lane_point"] = res["one_lane_point"]
    if "per_rank" in res:
        out["bubble_frac_max"] = round(res["bubble_frac_max"], 4)
        out["per_rank"] = res["per_rank"]
        for k in ("stage_cost_model_us", "stage_cost_spread", "slack", "host_issue_us_per_tick_max", "vocab_split",
                  "streams"):
            if k in res:
                out[k] = res[k]
    print(json.dumps(out), flush=True)
    MetricsWriter(args.metrics_out).write(event="bench", **out)
    return out


if __name__ == "__main__":
    main()

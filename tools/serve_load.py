#!/usr/bin/env python
"""Serving under load: the same Poisson arrival trace through ``ServingEngine`` on a single-GPU
``Generator`` (engine.continuous.SlotDecoder) and on the RCCL pipeline engine at world 1
(``PipelineGenerator`` + parallel.pp_slots: batched ragged admission, on-device token budgets,
graph-captured decode rounds).  One model, built once, serves both engines in turn.

Per engine: output tokens/s over the trace (first submission -> last completion), p50 / p99 of
TTFT (submission -> first token, queueing included) and of end-to-end latency, per-token decode
latency percentiles (the engine's histogram), and the most requests decoding together.

Reference: the reference's server answers one request per pool thread (Code/gRPC/server.py:14);
its generation loop is single-stream (combine_model_fp_updated.py:86-110).

    python tools/serve_load.py --model llama-2-7b --quant w8a8_smoothquant --requests 64 --rate 8 \
        --out gpurun_out/serve_load.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm.engine import Generator, SamplingParams  # noqa: E402
from edgellm.models.registry import load_model  # noqa: E402
from edgellm.serve.server import ServingEngine  # noqa: E402


def trace(n, rate, seed, plen, new, vocab=32000):
    """[(arrival_s, prompt ids, max_new)] with exponential inter-arrival times (rate req/s)."""
    rnd = random.Random(seed)
    t, out = 0.0, []
    for _ in range(n):
        t += rnd.expovariate(rate) if rate > 0 else 0.0
        L = rnd.randint(plen[0], plen[1])
        out.append((t, [rnd.randrange(3, vocab) for _ in range(L)], rnd.randint(new[0], new[1])))
    return out


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else float("nan")


def run(engine, tr, sp_kw):
    futs = []
    t0 = time.perf_counter()
    for at, ids, mx in tr:
        d = at - (time.perf_counter() - t0)
        if d > 0:
            time.sleep(d)
        futs.append(engine.submit(ids, SamplingParams(max_new_tokens=mx, **sp_kw)))
    res = [f.result(timeout=1800) for f in futs]
    wall = time.perf_counter() - t0
    toks = sum(len(r["tokens"]) for r in res)
    m = engine.metrics()
    return dict(requests=len(res), output_tokens=toks, wall_s=round(wall, 3), tokens_per_s=round(toks / wall, 1),
                ttft_p50_ms=round(pct([r["ttft_ms"] for r in res], 0.5), 2),
                ttft_p99_ms=round(pct([r["ttft_ms"] for r in res], 0.99), 2),
                latency_p50_ms=round(pct([r["latency_ms"] for r in res], 0.5), 1),
                latency_p99_ms=round(pct([r["latency_ms"] for r in res], 0.99), 1),
                token_ms_p50=m.get("p50_ms"), token_ms_p99=m.get("p99_ms"),
                max_concurrent=m.get("max_concurrent"), sessions=m.get("sessions"), decode_steps=m.get("decode_steps"))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-2-7b")
    ap.add_argument("--quant", default="w8a8_smoothquant")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--requests", type=int, default=64)
    ap.add_argument("--rate", type=float, default=8.0, help="mean arrivals per second (Poisson)")
    ap.add_argument("--prompt-len", default="32,256")
    ap.add_argument("--max-new", default="64,192")
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--max-seq", type=int, default=1024)
    ap.add_argument("--engines", default="generator,pipeline")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    model, tok, src = load_model(args.model, args.precision, args.quant, dev)
    pl = tuple(int(x) for x in args.prompt_len.split(","))
    nw = tuple(int(x) for x in args.max_new.split(","))
    V = model.cfg.vocab_size
    tr = trace(args.requests, args.rate, args.seed, pl, nw, V)
    sp_kw = dict(temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)   # Code/others/config.yaml:3-7
    rows = []
    for name in args.engines.split(","):
        if name == "generator":
            gen = Generator(model, max_batch=args.max_batch, max_seq=args.max_seq)
        else:
            from edgellm.parallel.pipeline import init_distributed
            from edgellm.parallel.pp_engine import PipelineGenerator
            for k, v in (("RANK", "0"), ("LOCAL_RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1")):
                os.environ.setdefault(k, v)
            if "MASTER_PORT" not in os.environ:
                import socket
                s = socket.socket()
                s.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s.getsockname()[1])
                s.close()
            init_distributed("nccl" if dev.type == "cuda" else "gloo")
            gen = PipelineGenerator(model, 0, 1, max_batch=args.max_batch, max_seq=args.max_seq)
        eng = ServingEngine(gen, tok, max_batch=args.max_batch)
        # warm-up: graphs and kernels of the first session outside the measured trace
        run(eng, trace(4, 0.0, args.seed + 1, pl, (8, 8), V), sp_kw)
        res = run(eng, tr, sp_kw)
        eng.close()
        row = dict(event="serve_load", engine=name, model=args.model, quant=args.quant, source=src,
                   rate_req_s=args.rate, prompt_len=list(pl), max_new=list(nw), max_batch=args.max_batch, **res)
        print(json.dumps(row), flush=True)
        rows.append(row)
        del eng, gen
        if dev.type == "cuda":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    if len(rows) == 2:
        a, b = rows
        print(json.dumps(dict(event="serve_load_ratio", pipeline_over_generator_tps=round(b["tokens_per_s"] / a["tokens_per_s"], 4),
                              ttft_p50_ratio=round(b["ttft_p50_ms"] / a["ttft_p50_ms"], 4),
                              ttft_p99_ratio=round(b["ttft_p99_ms"] / a["ttft_p99_ms"], 4))), flush=True)
    if args.out:
        with open(args.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Interleaved A/B of kernel knobs on the headline decode config (Llama-2-7B W8A8, lanes x 256
rows), building and calibrating the model ONCE: each round re-creates the LaneGenerator (the
knob is baked into the captured graphs) for every setting, so settings share the box, its clock
and its HBM state.

    python tools/lane_ab.py --knobs "none;decode_attn_persist=2;decode_attn_persist=3" --rounds 2

Prints one JSON line per (round, setting): tok/s, ms per step, p50 per-token latency.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from edgellm import ops  # noqa: E402
from edgellm.engine import Generator, SamplingParams  # noqa: E402
from edgellm.engine.generate import LaneGenerator  # noqa: E402


def measure(model, cfg, args, lanes: int) -> dict:
    B = args.micro_batch
    total_new = args.warmup + args.steps + 2
    max_seq = args.prompt_len + total_new + 8
    if lanes > 1:
        gen = LaneGenerator(model, lanes=lanes, max_batch=B, max_seq=max_seq, use_graphs=True)
        lanes_l = gen.lanes
    else:
        gen = Generator(model, max_batch=B, max_seq=max_seq, use_graphs=True)
        lanes_l = [gen]
    g = torch.Generator().manual_seed(args.seed)
    prompts = torch.randint(0, cfg.vocab_size, (B * lanes, args.prompt_len), generator=g).tolist()
    sp = SamplingParams(max_new_tokens=total_new, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)
    gen.start(prompts, sp, seed=args.seed)
    gen.step(args.warmup, record_latency=False)
    gen.precapture(args.steps + 1)
    torch.cuda.synchronize()
    n_ev = [len(x._run["events"]) for x in lanes_l]
    t0 = time.perf_counter()
    gen.step(args.steps, record_latency=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lat = []
    for x, n0 in zip(lanes_l, n_ev):
        ev = x._run["events"][n0:]
        lat += [ev[i - 1].elapsed_time(ev[i]) for i in range(1, len(ev))]
    lat.sort()
    del gen, lanes_l
    torch.cuda.empty_cache()
    return dict(tok_s=round(B * lanes * args.steps / dt, 1), ms_step=round(dt / args.steps * 1e3, 3),
                p50_ms=round(lat[len(lat) // 2], 3))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knobs", default="none", help="';'-separated settings; each is an EDGELLM_TUNE spec or 'none'")
    ap.add_argument("--reset", default="", help="EDGELLM_TUNE spec applied before every setting (defaults)")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--lanes", default="2", help="comma list of lane counts")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--micro-batch", type=int, default=256)
    ap.add_argument("--model", default="llama-2-7b")
    a = ap.parse_args()
    args = bench.parse(["--model", a.model, "--steps", str(a.steps), "--warmup", str(a.warmup),
                        "--micro-batch", str(a.micro_batch)])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg, model = bench.build(args, dev)
    ops.ext()
    settings = [s.strip() for s in a.knobs.split(";") if s.strip()]
    for r in range(a.rounds):
        for lanes in [int(x) for x in a.lanes.split(",")]:
            for s in settings:
                ops.apply_tune(a.reset)
                if s != "none":
                    ops.apply_tune(s)
                res = measure(model, cfg, args, lanes)
                print(json.dumps(dict(round=r, lanes=lanes, knobs=s, **res)), flush=True)
        ops.apply_tune(a.reset)


if __name__ == "__main__":
    main()

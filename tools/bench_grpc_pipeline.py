#!/usr/bin/env python
"""BASELINE config 1 — GPT-2-small layer-split into 2 stages over localhost gRPC on the CPU (the
"distributed edge" plumbing: the reference's gRPC demo carries only a time string,
Code/gRPC/time_service.proto:5-13; here the same transport carries activations).

Stage 0 (embedding + layers [0, 6)) runs in this process; stage 1 (layers [6, 12) + LM head +
sampler) is a gRPC server in a child process.  Random-init GPT-2-small weights (no checkpoints
offline), synthetic prompts.  Prints one JSON line: generated tok/s, p50 per-token latency and
the bytes shipped per decode step.

    python tools/bench_grpc_pipeline.py [--batch 4 --prompt-len 32 --new 32 --threads 4]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _stage_server(port_q, split, max_seq, threads):
    import torch
    torch.set_num_threads(threads)
    import edgellm  # noqa: F401
    from edgellm.models import build_model, get_config
    from edgellm.serve.stage_service import StageServer, serve_stage
    cfg = get_config("gpt2")
    model = build_model(cfg, dtype=torch.float32, first=split, last=cfg.num_layers, seed=0)
    server = serve_stage(StageServer(model, max_seq=max_seq), port=0, host="127.0.0.1")
    port_q.put(server.port)
    server.wait_for_termination()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--new", type=int, default=32)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--split", type=int, default=6)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    torch.set_num_threads(a.threads)
    import edgellm  # noqa: F401
    from edgellm.engine import Generator, SamplingParams
    from edgellm.models import build_model, get_config
    from edgellm.serve.stage_service import EdgePipeline, RemoteStage
    cfg = get_config("gpt2")
    max_seq = a.prompt_len + a.new + 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_stage_server, args=(q, a.split, max_seq, a.threads), daemon=True)
    proc.start()
    try:
        port = q.get(timeout=300)
        first = build_model(cfg, dtype=torch.float32, first=0, last=a.split, seed=0)
        remote = RemoteStage(f"127.0.0.1:{port}", timeout=60)
        pipe = EdgePipeline(first, [remote], max_seq=max_seq)
        g = torch.Generator().manual_seed(0)
        prompts = torch.randint(0, cfg.vocab_size, (a.batch, a.prompt_len), generator=g).tolist()
        sp = SamplingParams(max_new_tokens=a.new, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)
        pipe.generate(prompts, SamplingParams(max_new_tokens=4), seed=1)          # warm-up
        t0 = time.perf_counter()
        res = pipe.generate(prompts, sp, seed=2)
        wall = time.perf_counter() - t0
        # the same model unsplit, in-process (what the split costs)
        full = build_model(cfg, dtype=torch.float32, seed=0)
        ref = Generator(full, max_batch=a.batch, max_seq=max_seq).generate(prompts, sp, seed=2)
        step = sorted(res.step_ms)
        out = {
            "config": "GPT-2-small 2-stage layer split over localhost gRPC (CPU)",
            "split": [0, a.split, cfg.num_layers], "batch": a.batch, "prompt_len": a.prompt_len,
            "new_tokens": a.new, "threads_per_stage": a.threads,
            "tokens_per_s": round(res.num_generated / wall, 2),
            "p50_token_latency_ms": round(step[len(step) // 2], 3) if step else None,
            "prefill_s": round(res.prefill_s, 4),
            "hidden_bytes_per_decode_step": a.batch * cfg.hidden_size * 4,
            "unsplit_in_process_tokens_per_s": round(ref.tps_generated(), 2),
            "tokens_match_unsplit": res.tokens == ref.tokens,
            "data": "synthetic prompts, random-init GPT-2-small weights",
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
        remote.close()
    finally:
        proc.kill()


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Time-to-first-token of one prompt at batch 1 (the refiner / evaluator shape) and, under
rocprofv3 --kernel-trace, an isolated last prefill for tools/kernel_gaps.py: the final prefill
runs after a 200 ms idle gap, so ``kernel_gaps.py --window <ms>`` over the trace tail sees only it.

    python tools/prefill_profile.py --prompt-len 1024 [--quant w8a8_smoothquant|none]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from bench import build  # noqa: E402
from edgellm.engine import Generator, SamplingParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-2-7b")
    ap.add_argument("--quant", default="w8a8_smoothquant")
    ap.add_argument("--prompt-len", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    a.steps, a.warmup, a.lm_head, a.device = 4, 2, "bf16", None
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg, model = build(a, dev)
    g = torch.Generator().manual_seed(a.seed)
    prompt = torch.randint(0, cfg.vocab_size, (1, a.prompt_len), generator=g).tolist()
    sp = SamplingParams(max_new_tokens=2, temperature=0.7, top_k=50, top_p=0.9, repetition_penalty=1.1)
    gen = Generator(model, max_batch=1, max_seq=a.prompt_len + 16)
    ttft = []
    for r in range(a.reps + 1):
        torch.cuda.synchronize()
        if r == a.reps:
            time.sleep(0.2)                      # isolate the last prefill in a kernel trace
        t0 = time.perf_counter()
        gen.start(prompt, sp, seed=r)
        torch.cuda.synchronize()
        ttft.append((time.perf_counter() - t0) * 1e3)
    ttft = sorted(ttft[1:])
    print(json.dumps(dict(model=a.model, quant=a.quant, prompt_len=a.prompt_len, ttft_ms_p50=round(ttft[len(ttft) // 2], 3),
                          ttft_ms_min=round(ttft[0], 3), prefill_tok_s=round(a.prompt_len / ttft[len(ttft) // 2] * 1e3, 1))),
          flush=True)


if __name__ == "__main__":
    main()

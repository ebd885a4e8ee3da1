#!/usr/bin/env python
"""Reference point for the 256-row decode GEMMs: hipBLASLt's int8 GEMM (torch._int_mm, int32 out,
no epilogue) and bf16 GEMM (F.linear) at Llama-2-7B projection shapes, cache-cold, graph-timed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.bench_ops import timeit  # noqa: E402


def main(M=256):
    dev = torch.device("cuda:0")
    for name, (N, K) in {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096),
                         "down": (4096, 11008)}.items():
        ncopy = max(2, (1 << 30) // (N * K) + 1)
        ws = [torch.randint(-127, 128, (K, N), dtype=torch.int8, device=dev).t().contiguous().t() for _ in range(ncopy)]
        a = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        ctr = [0]

        def call():
            ctr[0] = (ctr[0] + 1) % ncopy
            return torch._int_mm(a, ws[ctr[0]])
        t = min(timeit(call, iters=10, per_graph=ncopy) for _ in range(3))
        wb = [torch.randn(N, K, device=dev).bfloat16() for _ in range(max(2, (1 << 30) // (2 * N * K) + 1))]
        x = torch.randn(M, K, device=dev).bfloat16()
        c2 = [0]

        def callb():
            c2[0] = (c2[0] + 1) % len(wb)
            return torch.nn.functional.linear(x, wb[c2[0]])
        tb = min(timeit(callb, iters=10, per_graph=len(wb)) for _ in range(3))
        print(dict(shape=name, M=M, N=N, K=K, int_mm_us=round(t, 2), int_mm_TBps=round(N * K / t / 1e6, 2),
                   bf16_us=round(tb, 2), bf16_TBps=round(2 * N * K / tb / 1e6, 2)), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 256)

"""LLM.int8 linear at prefill rows: the device path (ops/csrc/llmint8.hip, any rows, no host sync)
against the round-5 form (outlier columns by ``nonzero()`` on the host, torch GEMM for the outlier
part).  Llama-2-7B projection shapes, synthetic activations with a few outlier columns per
prompt; prints one JSON line per (shape, rows, outliers).

    python tools/llmint8_rows_ab.py [--iters 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402
from edgellm.models.layers import Linear  # noqa: E402
from edgellm.quant import LLMInt8Linear  # noqa: E402


def host_form(m: LLMInt8Linear, x2: torch.Tensor) -> torch.Tensor:
    """The round-5 prefill path, kept here only as the A/B baseline."""
    K, N = m.in_features, m.out_features
    cols = (x2.abs() > m.threshold).any(0).nonzero().flatten()
    w_scale = m.SCB / 127.0
    if cols.numel() > 0:
        x_in = x2.clone()
        x_in[:, cols] = 0
        w_out = (m.weight_i8[:, cols].float() * w_scale[:, None]).to(x2.dtype)
        out_o = x2[:, cols] @ w_out.t()
    else:
        x_in, out_o = x2, None
    q, s = ops.quant_per_token(x_in.contiguous())
    out = ops.w8a8_linear(q, s, m.w_packed, w_scale, m.bias, N, K)
    if out_o is not None:
        out = (out.float() + out_o.float()).to(out.dtype)
    return out


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
    for name, (K, N) in shapes.items():
        torch.manual_seed(0)
        lin = Linear(K, N, bias=False, device=dev)
        lin.weight.data.copy_(torch.randn(N, K, device=dev) * 0.02)
        m = LLMInt8Linear.from_float(lin)
        for M in (512, 2048):
            for n_out in (0, 8, 64):
                x = torch.randn(M, K, device=dev)
                if n_out:
                    x[torch.randint(0, M, (n_out,), device=dev), torch.randperm(K, device=dev)[:n_out]] = 9.0
                x = x.bfloat16()
                dev_out, host_out = m(x), host_form(m, x)
                err = ((dev_out.float() - host_out.float()).norm() / host_out.float().norm()).item()
                t_dev = timed(lambda: m(x), a.iters)
                t_host = timed(lambda: host_form(m, x), a.iters)
                print(json.dumps({"proj": name, "K": K, "N": N, "rows": M, "outlier_cols": n_out,
                                  "device_us": round(t_dev, 1), "host_sync_us": round(t_host, 1),
                                  "speedup": round(t_host / t_dev, 3), "rel_diff": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()

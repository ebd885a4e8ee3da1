#!/usr/bin/env python
"""Diagnose the x32 prefill GEMM's fragment / accumulator mapping with one-hot activations:
token t has a single 1 at k = t % K, so out[t][n] = W[n][t % K] * scales exactly.  Prints, per
(token % 32, column % 64) class, the fraction of wrong outputs, and where a wrong value came from."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402

dev = torch.device("cuda:0")
C = ops.ext()
M, N, K = 2048, 12288, 4096
t = torch.arange(M, device=dev)
x = torch.zeros(M, K, dtype=torch.int8, device=dev)
x[t, t % K] = 1
w = torch.randint(-100, 100, (N, K), dtype=torch.int8, device=dev)
sx = torch.ones(M, device=dev)
sw = torch.ones(N, device=dev)
wp = ops.pack_int8_weight(w)
for v in (0, 1):
    C.tune("prefill_x32", v, 0)
    C.tune("prefill_apack", 0, 0)
    out = C.w8a8_gemm(x, sx, wp, sw, None, N, K).float()
    ref = w[:, (t % K)].t().float()
    bad = (out - ref).abs() > 0.5
    print(f"x32={v}: wrong {bad.float().mean().item():.4f}", flush=True)
    if v and bad.any():
        cls = bad.view(M // 32, 32, N // 64, 64).float().mean((0, 2))
        print("wrong fraction by (token % 32) x (col % 64 in 8-col groups):")
        print(cls.view(32, 8, 8).mean(-1))
        r, c = torch.nonzero(bad)[0].tolist()
        val = out[r, c].item()
        cand = torch.nonzero((w[:, :].float() == val)[:, r % K]).flatten()[:8].tolist()
        print(f"first wrong out[{r}][{c}] = {val} (want {ref[r, c].item()}); W[n][{r % K}] == val at n = {cand}")
        cand2 = torch.nonzero(w[c].float() == val).flatten()[:8].tolist()
        print(f"  W[{c}][k] == val at k = {cand2}")
C.tune("prefill_x32", 0, 0)
C.tune("prefill_apack", 1, 0)

"""Diff pattern of the wreg 256-row kernel against ring2 over repeated calls (debug aid)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import edgellm  # noqa
from edgellm import ops

C = ops.ext()
dev = torch.device("cuda:0")
for (M, N, da, kind) in [(129, 12288, 4, "out"), (256, 12288, 4, "out"), (256, 4096, 6, "out"), (256, 22016, 4, "gluq"),
                         (200, 2048, 4, "gluq")]:
    K = 4096
    torch.manual_seed(M + N + da)
    qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
    sx = torch.rand(M, device=dev) * 0.01
    w = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
    sw = torch.rand(N, device=dev) * 0.01 + 1e-3
    wp = ops.pack_int8_weight(w)
    f = (lambda: C.w8a8_gemm_gluq(qx, sx, wp, sw, None, N, K)[0]) if kind == "gluq" else \
        (lambda: C.w8a8_gemm(qx, sx, wp, sw, None, N, K))
    C.tune("r256_wreg", 0, 0)
    want = f()
    C.tune("r256_wreg", da, 0)
    for it in range(4):
        got = f()
        torch.cuda.synchronize()
        bad = (got != want)
        n = int(bad.sum())
        if n:
            rows = bad.any(1).nonzero().flatten().tolist()
            cols = bad.any(0).nonzero().flatten().tolist()
            print(f"M={M} N={N} da={da} {kind} it={it}: {n} bad; rows {len(rows)} first {rows[:8]}; cols {len(cols)} "
                  f"first {cols[:8]} last {cols[-4:]}; col%128 set {sorted(set(c % 128 for c in cols))[:16]}", flush=True)
        else:
            print(f"M={M} N={N} da={da} {kind} it={it}: ok", flush=True)
    C.tune("r256_wreg", 0, 0)

"""Run one 128-row grouped-scale split-K GEMV (Llama-2-7B o or down) in a loop, for rocprofv3 --pmc.

    python tools/o_probe.py --shape o --ring 0|2 [--cfg C] [--iters N]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
import edgellm  # noqa: E402,F401
from edgellm import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="o", choices=["o", "down"])
ap.add_argument("--ring", type=int, default=0)
ap.add_argument("--cfg", type=int, default=0)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
N, K = {"o": (4096, 4096), "down": (4096, 11008)}[a.shape]
M, dev = 128, "cuda"
C = ops.ext()
C.tune("gemv_ring", a.ring, 0)
C.tune("ring2_cfg", a.cfg, 1)
ncopy = (1 << 30) // (N * K) + 1
wps = [ops.pack_int8_weight(torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)) for _ in range(ncopy)]
sw = torch.rand(N, device=dev) * 0.01
qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
sx = torch.rand(K // 64, M, device=dev) * 0.01
for i in range(a.iters):
    C.w8a8_gemm_splitk(qx, sx, wps[i % ncopy], sw, None, N, K, 4)
torch.cuda.synchronize()
print("ok", a.shape, a.ring, a.cfg)

if os.environ.get("O_PROBE_TIME"):
    from bench_ops import timeit  # noqa: E402
    for sh, (N, K) in {"o": (4096, 4096), "down": (4096, 11008)}.items():
        ncopy = (1 << 30) // (N * K) + 1
        wps = [ops.pack_int8_weight(torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)) for _ in range(ncopy)]
        sw = torch.rand(N, device=dev) * 0.01
        qx = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        sx = torch.rand(K // 64, M, device=dev) * 0.01
        for ring, cfg, S in [(0, 0, 4), (2, 1, 4), (2, 5, 4), (2, 6, 4), (2, 4, 4)]:
            if ring == 0 and S != 4:
                continue
            C.tune("gemv_ring", ring, 0)
            C.tune("ring2_cfg", cfg, 1)
            ctr = [0]

            def call():
                ctr[0] = (ctr[0] + 1) % ncopy
                return C.w8a8_gemm_splitk(qx, sx, wps[ctr[0]], sw, None, N, K, S)
            t = min(timeit(call, iters=10, per_graph=ncopy) for _ in range(3))
            print(dict(shape=sh, ring=ring, cfg=cfg, S=S, us=round(t, 2)), flush=True)
        # unsplit (EPI_OUT, bf16 out) on the same grouped-scale input: isolates the fp32 slice writes
        C.tune("gemv_ring", 0, 0)
        ctr = [0]

        def call_out():
            ctr[0] = (ctr[0] + 1) % ncopy
            return C.w8a8_gemm(qx, sx, wps[ctr[0]], sw, None, N, K)
        try:
            t = min(timeit(call_out, iters=10, per_graph=ncopy) for _ in range(3))
            print(dict(shape=sh, ring=0, cfg=0, S=1, epi="out_bf16", us=round(t, 2)), flush=True)
        except RuntimeError as e:      # no unsplit 128-row kernel for this K (down: 172 k-tiles)
            print(dict(shape=sh, S=1, epi="out_bf16", skipped=str(e)[:80]), flush=True)
    C.tune("gemv_ring", 2, 0)
    C.tune("ring2_cfg", 0, 0)

#!/bin/bash
# Round 2 (w): decoupled-depth ring GEMV (ring2) — exactness vs the LDS-staged kernel, then timing.
set -o pipefail
mkdir -p gpurun_out/r2w
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "ring" > gpurun_out/r2w/tests.log 2>&1 || { tail -30 gpurun_out/r2w/tests.log; exit 1; }
tail -1 gpurun_out/r2w/tests.log
timeout -k 10 300 python -u tools/bench_ops.py --only ring --out gpurun_out/r2w/ring.json > gpurun_out/r2w/ring.log 2>&1 || { tail -5 gpurun_out/r2w/ring.log; exit 1; }
grep "'op'" gpurun_out/r2w/ring.log

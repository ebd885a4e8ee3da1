#!/bin/bash
# Round 2 (x): whole-line activation pieces (ring form 3) — exactness, timing, ingest microbench.
set -o pipefail
mkdir -p gpurun_out/r2x /tmp/ib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "ring" > gpurun_out/r2x/tests.log 2>&1 || { tail -30 gpurun_out/r2x/tests.log; exit 1; }
tail -1 gpurun_out/r2x/tests.log
timeout -k 10 300 python -u tools/bench_ops.py --only ring --out gpurun_out/r2x/ring.json > gpurun_out/r2x/ring.log 2>&1 || { tail -5 gpurun_out/r2x/ring.log; exit 1; }
grep "'op'" gpurun_out/r2x/ring.log
exit 0
timeout -k 10 120 /tmp/ib/ingest_bw > gpurun_out/r2x/ingest.csv 2>&1 || exit 1
grep "^2,\|^3," gpurun_out/r2x/ingest.csv | grep ",256,8,"

#!/bin/bash
# Round 2 (p): prefill GEMM final-form tests + sweep + bench, then batch-1 GEMV sweep.
set -o pipefail
bash tools/gpu_r2o.sh || exit 1
timeout -k 10 400 python -u tools/bench_ops.py --only m1 --out gpurun_out/r2o/m1.json > gpurun_out/r2o/m1.log 2>&1 || { tail -20 gpurun_out/r2o/m1.log; exit 1; }
grep "'op'" gpurun_out/r2o/m1.log

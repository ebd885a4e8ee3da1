#!/bin/bash
# Round 2 (z): ring2 grouped-scale split-K (o / down) exactness + timing; pipeline HeadInfer failure triage.
set -o pipefail
mkdir -p gpurun_out/r2z
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "ring or rows128" > gpurun_out/r2z/tests.log 2>&1 || { tail -30 gpurun_out/r2z/tests.log; exit 1; }
tail -1 gpurun_out/r2z/tests.log
timeout -k 10 300 python -u tools/bench_ops.py --only ring --out gpurun_out/r2z/ring.json > gpurun_out/r2z/ring.log 2>&1 || { tail -5 gpurun_out/r2z/ring.log; exit 1; }
grep "'op'" gpurun_out/r2z/ring.log
for v in "" "EDGELLM_OFFLOAD_SYNC=1" "EDGELLM_HEADINFER_COPY_MODE=2"; do
  env $v timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_pipeline_gpu.py -k "headinfer" > gpurun_out/r2z/hi.log 2>&1; echo "[$v] rc=$? $(tail -1 gpurun_out/r2z/hi.log)"
done

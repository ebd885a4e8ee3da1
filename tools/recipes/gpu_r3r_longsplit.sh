#!/bin/bash
# 256-row down-projection split-K slices (ring2_256_splits=2,L): default 4 vs 2 vs 8, in-model, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rows256_gpu.py \
  -k slice_counts > gpurun_out/r3r_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
: > gpurun_out/r3r_ab.jsonl
for r in 1 2; do
  for L in 4 2 8; do
    EDGELLM_TUNE="ring2_256_splits=2,$L" timeout -k 10 240 python bench.py --steps 20 --warmup 5 --latency-point off \
      > gpurun_out/r3r_b.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r3r_b.log; exit 1; }
    grep '^{' gpurun_out/r3r_b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());d['ab_label']='down slices $L';print(json.dumps(d))" >> gpurun_out/r3r_ab.jsonl
    python -c "import json;d=[json.loads(l) for l in open('gpurun_out/r3r_ab.jsonl')][-1];print(d['ab_label'],d['value'],d.get('p50_token_latency_ms'))"
  done
done
echo DONE

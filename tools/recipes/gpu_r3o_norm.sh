#!/bin/bash
# Batch-1 norm-in-GEMV-prologue: numerics tests, interleaved A/B (gemv_norm=1 / 0), kernel table.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_gpu.py \
  -k "gemv_norm or defers_norms" > gpurun_out/${TAG:-r3o}_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/${TAG:-r3o}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG:-r3o}_tests.log
: > gpurun_out/${TAG:-r3o}_ab.jsonl
for r in 1 2; do
  for k in 1 0; do
    EDGELLM_TUNE="gemv_norm=$k" timeout -k 10 240 python bench.py --micro-batch 1 --steps 64 --warmup 8 \
      --latency-point off > gpurun_out/${TAG:-r3o}_b.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG:-r3o}_b.log; exit 1; }
    grep '^{' gpurun_out/${TAG:-r3o}_b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());d['ab_label']='batch1 gemv_norm=$k';print(json.dumps(d))" >> gpurun_out/${TAG:-r3o}_ab.jsonl
    python -c "import json;d=[json.loads(l) for l in open('gpurun_out/${TAG:-r3o}_ab.jsonl')][-1];print(d['ab_label'],d['value'],d.get('p50_token_latency_ms'),d.get('p90_token_latency_ms'))"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG:-r3o} -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --micro-batch 1 --steps 64 --warmup 8 --latency-point off > $GRAFT_REPO_ROOT/gpurun_out/${TAG:-r3o}_prof.log 2>&1 \
  || { echo PROF_FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/${TAG:-r3o}_prof.log; exit 1; }
echo DONE

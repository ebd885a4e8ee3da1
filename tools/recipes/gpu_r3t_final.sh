#!/bin/bash
# Round-3 final validation on the current kernels: GPU test suite, smoke, default bench (20 steps),
# bf16 bench, and the reference's batch-1 single-model loop (Llama-3.2-1B, bf16 vs W8A8).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
D=gpurun_out/r3t
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gputests.log 2>&1 \
  || { echo GPUTESTS_FAILED; tail -40 $D/gputests.log; exit 1; }
tail -2 $D/gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $D/smoke.log 2>&1 \
  || { echo SMOKE_FAILED; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 $D/bench.log; exit 1; }
grep '^{' $D/bench.log > $D/bench.jsonl
timeout -k 10 300 python bench.py --quant none --steps 20 --warmup 5 --latency-point off > $D/bench_bf16.log 2>&1 \
  || { echo BF16_FAILED; tail -20 $D/bench_bf16.log; exit 1; }
grep '^{' $D/bench_bf16.log >> $D/bench.jsonl
python -c "
import json
for l in open('$D/bench.jsonl'):
    d=json.loads(l); print(d['config'].get('quant'), d['value'], d.get('p50_token_latency_ms'), json.dumps(d.get('latency_point'))[:300])"
echo DONE

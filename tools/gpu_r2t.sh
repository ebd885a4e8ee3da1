#!/bin/bash
# Round 2 (t): where batch-1 decode time goes on a 1B model — kernel durations vs inter-kernel gaps.
set -o pipefail
mkdir -p gpurun_out/r2t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for mode in w8a8_smoothquant none; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2t/$mode -- python3 tools/bench_reference_config.py --models llama-3.2-1b --modes $mode --repeats 1 > gpurun_out/r2t/$mode.log 2>&1 || { tail -5 gpurun_out/r2t/$mode.log; exit 1; }
  f=$(ls gpurun_out/r2t/$mode/*/*kernel_trace.csv | head -1)
  echo "== $mode"; grep -h '^{' gpurun_out/r2t/$mode.log | cut -c1-300
  python3 tools/kernel_gaps.py $f --window 40 --top 14
done

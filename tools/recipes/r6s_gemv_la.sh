# Round 6: cache-cold GEMV microbenchmarks (M = 1-64) with the lookahead for odd k ranges at
# MB <= 4 (this tree) vs without it (ab_old/), same box, alternating
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6s; mkdir -p $D
cd $R
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py -k "gemv or w8a8 or norm or linear" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cd $R/ab_old; else cd $R; fi
    timeout -k 10 300 python3 tools/bench_ops.py --only gemv,grouped --no-sweep > $D/ops_${v}_$i.log 2>&1 || { tail -20 $D/ops_${v}_$i.log; exit 1; }
  done
done

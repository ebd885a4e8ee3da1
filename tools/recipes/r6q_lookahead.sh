# Round 6: batch-1 A/B of the down-projection GEMV lookahead (ab_old/ = the tree before it, same box,
# alternating), plus the bit-exact gemv-norm tests on the new build
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6q; mkdir -p $D
cd $R
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py -k "gemv or w8a8 or norm or linear" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for i in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then cd $R/ab_old; else cd $R; fi
    timeout -k 10 300 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b_${v}_$i.log 2>&1 || { tail -20 $D/b_${v}_$i.log; exit 1; }
    echo "$v $i $(grep '^{' $D/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("p50_ms"), d["value"])')"
  done
done

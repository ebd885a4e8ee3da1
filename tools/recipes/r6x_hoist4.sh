# Round 6: the norm-prologue load hoist widened to NCH x SMAX <= 4 (K = 2048 with 3-4 slices:
# Llama-3.2-1B) vs ab_old/ (before), batch-1 Llama-3.2-1B and Llama-2-7B W8A8, alternating
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6x; mkdir -p $D
cd $R
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py -k "gemv or w8a8 or norm or linear" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for m in llama-3.2-1b llama-2-7b; do
for i in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then cd $R/ab_old; else cd $R; fi
    timeout -k 10 300 python3 bench.py --model $m --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b_${m}_${v}_$i.log 2>&1 || { tail -20 $D/b_${m}_${v}_$i.log; exit 1; }
    echo "$m $v $i $(grep '^{' $D/b_${m}_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
done

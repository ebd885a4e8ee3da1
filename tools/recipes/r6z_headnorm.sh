# Round 6: final RMSNorm in the LM-head GEMV prologue — the whole GPU suite, then batch-1 W8A8 Llama-2-7B
# (ab_old/: before it; the other round-6 changes there are neutral at 7B) and Llama-3.2-1B bf16
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6z; mkdir -p $D
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cd $R/ab_old; else cd $R; fi
    timeout -k 10 300 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b_7b_${v}_$i.log 2>&1 || { tail -20 $D/b_7b_${v}_$i.log; exit 1; }
    echo "7b-w8a8 $v $i $(grep '^{' $D/b_7b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done

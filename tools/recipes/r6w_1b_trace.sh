# Round 6: kernel traces of the Llama-3.2-1B batch-1 decode step, W8A8 and bf16
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6w; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
for q in w8a8_smoothquant none; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_$q -o run -- python3 $R/bench.py --model llama-3.2-1b --quant $q --micro-batch 1 --lanes 1 --steps 16 --warmup 4 --latency-point off > $D/prof_$q.log 2>&1 || { tail -20 $D/prof_$q.log; exit 1; }
  grep '^{' $D/prof_$q.log | cut -c1-250
done

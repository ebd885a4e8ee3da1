# Round 6: norm fusion at 2-4 decode rows now that the prologue loads issue first
# (EDGELLM_NORM_FUSE_ROWS 1 = default vs 4), Llama-2-7B W8A8 and Llama-3.2-1B bf16 at 2 and 4 rows
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6ad; mkdir -p $D
for cfg in "llama-2-7b w8a8_smoothquant 4" "llama-2-7b w8a8_smoothquant 2" "llama-3.2-1b none 4"; do
  set -- $cfg
  for i in 1 2; do
    for r in 1 4; do
      EDGELLM_NORM_FUSE_ROWS=$r timeout -k 10 300 python3 bench.py --model $1 --quant $2 --micro-batch $3 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b_${1}_${2}_${3}_r${r}_${i}.log 2>&1 || { tail -20 $D/b_${1}_${2}_${3}_r${r}_${i}.log; exit 1; }
      echo "$1 $2 rows=$3 fuse_rows=$r run=$i $(grep '^{' $D/b_${1}_${2}_${3}_r${r}_${i}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
    done
  done
done

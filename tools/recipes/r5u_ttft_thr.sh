# 32K TTFT: exact online softmax vs the deferred max (thr 8), alternating, same box
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5u; mkdir -p $D
for r in 1 2; do
for t in "0,0" "0,8"; do
  EDGELLM_TUNE="prefill_fa_sm=$t" timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft_${t/,/_}_$r.log 2>&1 || exit $?
done
done

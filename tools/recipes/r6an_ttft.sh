# Round 6 final tree: the 32K-token Llama-3-8B W8A8 TTFT (verdict item 7), three repetitions x 2
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6an; mkdir -p $D
for i in 1 2; do
  timeout -k 10 400 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft_$i.log 2>&1 || { tail -20 $D/ttft_$i.log; exit 1; }
  grep -E "ttft|TTFT|^\{" $D/ttft_$i.log | tail -3 | cut -c1-300
done

# flash prefill: asm vs builtin transposed V reads on ONE box (interleaved kernel A/B, alternating 32K TTFT)
# (ran on the A/B build with tune key prefill_fa_tr; the knob and the builtin form were removed after this measurement)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5za; mkdir -p $D
timeout -k 10 600 python3 tools/fa_ab.py --knob tr --rounds 6 --out $D/fa_tr_ab.json > $D/fa_ab.log 2>&1 || exit $?
for r in 1 2; do
for t in 1 0; do
  EDGELLM_TUNE="prefill_fa_tr=$t" timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft_tr${t}_$r.log 2>&1 || exit $?
done
done

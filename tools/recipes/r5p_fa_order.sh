# flash-prefill workgroup order: numerics (bit-identical orders), interleaved A/B, 32K TTFT per order
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5p; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/fa_ab.py --knob order --rounds 5 --out $D/fa_order_ab.json > $D/fa_ab.log 2>&1 || exit $?
for o in 1 0; do
  EDGELLM_TUNE="prefill_fa_order=$o" timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft_order$o.log 2>&1 || exit $?
done

# flash prefill: DMA look-ahead 3 tiles (5-slot ring) vs 2 (numerics, interleaved A/B, alternating 32K TTFT)
# (ran on the A/B build with tune key prefill_fa_la; the 3-tile form was removed after this measurement)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5ze; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/fa_ab.py --knob la --rounds 6 --out $D/fa_la_ab.json > $D/fa_ab.log 2>&1 || exit $?
for r in 1 2; do
for v in 3 2; do
  EDGELLM_TUNE="prefill_fa_la=$v" timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft_la${v}_$r.log 2>&1 || exit $?
done
done

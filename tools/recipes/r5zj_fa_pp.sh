# flash prefill: pending P in swapping register sets vs copied per tile (numerics incl. odd / even tile
# (ran on the A/B build with tune key prefill_fa_pp; the copy form was removed after this measurement)
# counts, interleaved A/B, alternating 32K TTFT)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zj; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/fa_ab.py --knob pp --rounds 6 --out $D/fa_pp_ab.json > $D/fa_ab.log 2>&1 || exit $?
for r in 1 2; do
for v in 1 0; do
  EDGELLM_TUNE="prefill_fa_pp=$v" timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft_pp${v}_$r.log 2>&1 || exit $?
done
done

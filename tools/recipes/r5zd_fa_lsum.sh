# flash prefill: softmax row sums on the MFMA vs the VALU (numerics, interleaved A/B, alternating 32K TTFT)
# (ran on the A/B build with tune key prefill_fa_lsum; the MFMA row-sum form was removed after this measurement)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zd; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/fa_ab.py --knob lsum --rounds 6 --out $D/fa_lsum_ab.json > $D/fa_ab.log 2>&1 || exit $?
for r in 1 2; do
for v in 1 0; do
  EDGELLM_TUNE="prefill_fa_lsum=$v" timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft_ls${v}_$r.log 2>&1 || exit $?
done
done

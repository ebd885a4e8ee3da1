# prefill gate_up with the SwiGLU in the x32 epilogue: numerics, then 32K TTFT alternating fused / unfused on one box
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zc; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_prefill_x32_gpu.py tests/test_model_gpu.py tests/test_decode_numerics_gpu.py -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
for r in 1 2; do
for v in 1 0; do
  EDGELLM_PREFILL_GLU=$v timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft_glu${v}_$r.log 2>&1 || exit $?
done
done

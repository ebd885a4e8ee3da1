# flash prefill: transposed V reads in inline asm (no compiler vmcnt(0) before P.V); numerics, speed, 32K TTFT
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5y; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/fa_ab.py --knob stagger --rounds 4 --out $D/fa_stagger_ab.json > $D/fa_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft.log 2>&1 || exit $?

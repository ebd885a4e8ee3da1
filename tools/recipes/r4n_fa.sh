# Round-4: flash-prefill kernel with hoisted LDS offsets and two V steps in flight: tests, A/B, 32K TTFT
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4n; mkdir -p $D
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "prefill_attention" > $D/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/bench_ops.py --only prefill --out $D/ab_fa.json > $D/ab_fa.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft32k.log 2>&1 || exit $?

# Round-4: staggered-DMA x32 prefill GEMMs (tests + A/B), lanes-2 latency point
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4k; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_prefill_x32_gpu.py tests/test_bf16_x32_gpu.py > $D/x32_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_ops.py --only stg --out $D/ab_stg.json > $D/ab_stg.log 2>&1 || exit $?

# Round-4: pipeline GPU test triage, x32 tests + A/B (int8 and bf16), default bench
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4g; mkdir -p $D
timeout -k 10 120 python3 tools/determinism_probe.py > $D/determinism.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py > $D/pipeline_tests.log 2>&1
timeout -k 10 120 python3 tools/x32_debug.py > $D/x32_debug.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_prefill_x32_gpu.py tests/test_bf16_x32_gpu.py > $D/x32_tests.log 2>&1
timeout -k 10 600 python3 tools/bench_ops.py --only x32,bf16x32 --out $D/ab_x32.json > $D/ab_x32.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?

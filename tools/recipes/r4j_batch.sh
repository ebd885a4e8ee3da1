# Round-4: pipeline GPU tests after the staging fix, prefill ring-depth A/B, then r4h (lanes, prefetch, rehearsal)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4j; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py tests/test_rccl_gpu.py > $D/pipeline_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_ops.py --only stages --out $D/ab_stages.json > $D/ab_stages.log 2>&1 || exit $?
bash tools/recipes/r4h_batch.sh

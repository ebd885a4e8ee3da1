set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r3g}
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rows256_gpu.py > $D/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_ops.py --only rows256 --out $D/rows256.json > $D/rows256.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --lanes 1 --micro-batch 256 --latency-point off > $D/bench_1x256.log 2>&1
rc=$?
tail -n 2 $D/tests.log; grep op $D/rows256.log; grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' $D/bench*.log
exit $rc

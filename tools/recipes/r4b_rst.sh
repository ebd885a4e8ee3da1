# restaged-epilogue correctness + A/B on the 256-row decode GEMMs
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4b; mkdir -p $D
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rows256_gpu.py > $D/t.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_ops.py --only rst --out $D/ab_rst.json > $D/ab.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/bench.log 2>&1

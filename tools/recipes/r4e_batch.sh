# Round-4 validation batch: GPU tests (after pruning), x32 prefill GEMM A/B, 256-row k-rotation A/B,
# batch-1 weight-prefetch A/B, default bench, then the 1-GPU 2-rank gloo pipeline rehearsal.
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4e; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $D/gputest.log 2>&1 || exit $?
timeout -k 10 500 python3 tools/bench_ops.py --only x32,rot --out $D/ab.json > $D/ab.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?

# Round-4: 16-byte score loads in the split sampler's top-k chunk kernel (tune sample_vec) —
# sampler tests, kernel A/B and batch-1 A/B, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4sv; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "sample" > $D/tests.log 2>&1 || exit $?
for N in 1 0 1 0; do
  timeout -k 10 300 python3 tools/bench_ops.py --only sample --no-sweep --tune sample_vec=$N > $D/ops_v$N.$RANDOM.log 2>&1 || exit $?
done
for N in 1 0 1 0; do
  EDGELLM_TUNE="sample_vec=$N" timeout -k 10 400 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 \
    --latency-point off > $D/b1_v$N.$RANDOM.log 2>&1 || exit $?
done

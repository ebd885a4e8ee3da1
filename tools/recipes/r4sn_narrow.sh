# Round-4: top-k merge narrowing cap (tune sample_narrow: 0 = FCAP 256, v = max(top_k, v * top_k)):
# sampler tests under v = 2, sampler kernel A/B, batch-1 A/B (interleaved)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4sn; mkdir -p $D
EDGELLM_TUNE="sample_narrow=2" timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "sample" > $D/tests_n2.log 2>&1 || exit $?
for N in 0 2 3 0 2 3; do
  timeout -k 10 300 python3 tools/bench_ops.py --only sample --no-sweep --tune sample_narrow=$N > $D/ops_n$N.$RANDOM.log 2>&1 || exit $?
done
for N in 0 2 0 2; do
  EDGELLM_TUNE="sample_narrow=$N" timeout -k 10 400 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 \
    --latency-point off > $D/b1_n$N.$RANDOM.log 2>&1 || exit $?
done

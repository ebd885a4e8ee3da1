# Round-4: 16-byte score loads in the argmax chunk kernel too (greedy / full-vocab sampling):
# sampler tests, kernel A/B, then the full validation recipe
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4sx; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "sample" > $D/tests.log 2>&1 || exit $?
for N in 1 0 1 0; do
  timeout -k 10 300 python3 tools/bench_ops.py --only sample --no-sweep --tune sample_vec=$N > $D/ops_v$N.$RANDOM.log 2>&1 || exit $?
done
bash tools/recipes/r4x_validate.sh

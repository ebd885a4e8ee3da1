# Round 5: gemm_i8 consolidation (ldsa / tiled / one-ring kernels retired: 65-128 rows on ring2,
# ragged prefill on the 128 x 256 ring kernel; prefill GEMMs in gemm_i8_prefill.hip) — kernel,
# fused-path, model and numerics suites, then the default bench and the 65-128-row GLU timings
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5k; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_prefill_x32_gpu.py tests/test_rows256_gpu.py tests/test_model_gpu.py tests/test_decode_numerics_gpu.py tests/test_bf16_ring_gpu.py -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_ops.py --only glu,gemv --no-sweep --out $D/ops.json > $D/ops.log 2>&1 || exit $?

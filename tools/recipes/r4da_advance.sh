# Round-4: one-launch decode bookkeeping (ops.decode_advance) — tests, batch-1 points
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4da; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_cogen_gpu.py tests/test_model_gpu.py > $D/tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bench_reference_config.py --models llama-3.2-1b,pythia-1b --modes none,w8a8_smoothquant --repeats 3 > $D/refcfg.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $D/bench.log 2>&1 || exit $?

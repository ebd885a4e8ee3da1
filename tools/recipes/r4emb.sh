# Round-4: first norm deferred over an fp32 embedding slice (batch 1) — tests and batch-1 points
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4emb; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_cogen_gpu.py tests/test_kernels_gpu.py > $D/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b1.log 2>&1 || exit $?
timeout -k 10 900 python3 tools/bench_reference_config.py --modes none,w8a8_smoothquant --repeats 3 > $D/refcfg.log 2>&1 || exit $?

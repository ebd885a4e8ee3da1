set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 150 python -u -m pytest "tests/test_pipeline_gpu.py::test_pipeline_gpu_headinfer_chunked" -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r2c/pytest_hi.log 2>&1; echo pytest_hi rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2c/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2c/bench.log
EDGELLM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --micro-batch 64 > gpurun_out/r2c/bench_gloo2.log 2>&1 || exit $?
tail -1 gpurun_out/r2c/bench_gloo2.log

set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_headinfer.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2b/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r2b/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2b/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2b/bench.log
EDGELLM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --micro-batch 64 > gpurun_out/r2b/bench_gloo2.log 2>&1 || exit $?
tail -1 gpurun_out/r2b/bench_gloo2.log

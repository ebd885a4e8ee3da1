set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 300 python -u -m pytest tests/test_kv_int8.py tests/test_pipeline_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2d/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r2d/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2d/bench_kv8.log 2>&1 || exit $?
tail -1 gpurun_out/r2d/bench_kv8.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --kv-dtype bf16 --latency-point off > gpurun_out/r2d/bench_kv16.log 2>&1 || exit $?
tail -1 gpurun_out/r2d/bench_kv16.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2d/prof -o kv8 -- python3 bench.py --steps 16 --warmup 4 --latency-point off > gpurun_out/r2d/prof.log 2>&1; echo prof rc=$?

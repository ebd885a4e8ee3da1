# Round 6 baseline: the changed GPU tests, smoke, the default bench and its kernel trace
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6a; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_fp16_gpu.py tests/test_kv_int8.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench.py --steps 10 --warmup 3 --latency-point off --lanes 1 > $D/prof.log 2>&1 || exit $?

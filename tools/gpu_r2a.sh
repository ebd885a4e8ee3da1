set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1; echo pytest rc=$?; tail -3 gpurun_out/r2a/pytest.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r2a/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2a/bench.log
timeout -k 10 240 python bench.py --lanes 1 --steps 20 --warmup 5 > gpurun_out/r2a/bench_l1.log 2>&1 || exit $?
tail -1 gpurun_out/r2a/bench_l1.log
timeout -k 10 240 python bench.py --lanes 1 --micro-batch 1 --steps 64 --warmup 5 > gpurun_out/r2a/bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/r2a/bench_b1.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2a/prof -o def -- python3 bench.py --steps 16 --warmup 4 > gpurun_out/r2a/prof.log 2>&1; echo prof rc=$?

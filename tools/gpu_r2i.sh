set -o pipefail
mkdir -p gpurun_out/r2i
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -q -x --timeout 100 --timeout-method thread -k "rows128 or ring or gluq" > gpurun_out/r2i/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/r2i/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --latency-point off > gpurun_out/r2i/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2i/bench.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lanes 1 --latency-point off > gpurun_out/r2i/bench_l1.log 2>&1 || exit $?
tail -1 gpurun_out/r2i/bench_l1.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2i/prof -o ring -- python3 bench.py --steps 16 --warmup 4 --latency-point off > gpurun_out/r2i/prof.log 2>&1; echo prof rc=$?

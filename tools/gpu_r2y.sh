#!/bin/bash
# Round 2 (y): re-entry check after the container rebuild — full GPU tests, default bench, latency points, kernel stats.
set -o pipefail
mkdir -p gpurun_out/r2y2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2y2/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r2y2/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2y2/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2y2/bench.log
timeout -k 10 240 python bench.py --lanes 1 --steps 20 --warmup 5 --latency-point off > gpurun_out/r2y2/bench_l1.log 2>&1 || exit $?
tail -1 gpurun_out/r2y2/bench_l1.log
EDGELLM_TUNE="ring2_cfg=5,1" timeout -k 10 240 python bench.py --steps 20 --warmup 5 --latency-point off > gpurun_out/r2y2/bench_ring1.log 2>&1 || exit $?
tail -1 gpurun_out/r2y2/bench_ring1.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2y2/prof -o def -- python3 bench.py --steps 16 --warmup 4 --latency-point off > gpurun_out/r2y2/prof.log 2>&1; echo prof rc=$?

#!/bin/bash
# Round 2 final: full GPU suite, driver smoke, default bench, kernel-trace profile of the default bench.
set -o pipefail
mkdir -p gpurun_out/r2final2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2final2/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/r2final2/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2final2/smoke.log 2>&1 || { tail -5 gpurun_out/r2final2/smoke.log; exit 1; }
tail -1 gpurun_out/r2final2/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r2final2/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2final2/bench.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2final2/prof -o def -- python3 bench.py --steps 16 --warmup 4 --latency-point off > gpurun_out/r2final2/prof.log 2>&1; echo prof rc=$?

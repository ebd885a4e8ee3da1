# Round-4 final validation: full GPU suite, smoke, default bench (one lane point + batch-1 included)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4x; mkdir -p $D
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $D/gputest.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $D/bench.log 2>&1 || exit $?

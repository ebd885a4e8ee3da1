# Round 6: the whole GPU suite, smoke(), and the default bench (the driver's round-end sequence)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6f; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?

# exact final tree: full GPU suite, smoke, default bench, 32K TTFT
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zk; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft.log 2>&1 || exit $?

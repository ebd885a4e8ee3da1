# Round-4 validation: GPU tests, default bench (2 x 256) + rocprof stats, x32 A/B, prefill PMC, 32K TTFT
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4l; mkdir -p $D
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $D/gputest.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/prof.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_ops.py --only x32 --out $D/ab_x32.json > $D/ab_x32.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 3 > $D/ttft32k.log 2>&1 || exit $?
bash tools/recipes/pmc_prefill_gemm_r4.sh > $D/pmc.log 2>&1 || exit $?

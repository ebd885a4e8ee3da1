# kernel table of the default bench with the final round-5 tree
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zg; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --latency-point off > $GRAFT_REPO_ROOT/$D/bench.log 2>&1 || exit $?

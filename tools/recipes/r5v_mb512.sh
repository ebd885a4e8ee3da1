# one 512-row micro-batch per step vs the 2 x 256 default (same box); kernel trace of the 512-row step
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5v; mkdir -p $D
timeout -k 10 400 python3 bench.py --micro-batch 512 --lanes 1 --steps 20 --warmup 5 --latency-point off > $D/mb512.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/default.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --micro-batch 384 --lanes 1 --steps 20 --warmup 5 --latency-point off > $D/mb384.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --micro-batch 512 --lanes 1 --steps 10 --warmup 3 --latency-point off > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 || exit $?

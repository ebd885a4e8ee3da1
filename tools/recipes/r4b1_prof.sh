# Round-4: kernel table of Llama-2-7B W8A8 at batch 1 (bench.py --micro-batch 1 --lanes 1)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4b1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/prof.log 2>&1 || exit $?

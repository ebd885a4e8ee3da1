# Round-4: batch-1 Llama-2-7B W8A8 kernel table and last-step kernel sequence after the
# sampler-fused decode bookkeeping
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4sb; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/prof.log 2>&1 || exit $?

# Round-4 final-state kernel tables: bench default (2 x 256; the tracer serialises the lanes) and
# batch 1 (Llama-2-7B W8A8)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4fp; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/def -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/def.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/b1 -o run --output-format csv -- python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b1.log 2>&1 || exit $?

# Round 6: kernel trace of the batch-1 W8A8 decode step on the final round-6 tree
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6at; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 $R/bench.py --micro-batch 1 --lanes 1 --steps 8 --warmup 3 --latency-point off > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
grep '^{' $D/prof.log | cut -c1-200

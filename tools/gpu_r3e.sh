set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r3e}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
EDGELLM_DEC256_SCALES=token timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 32 --warmup 4 --lanes 1 --micro-batch 256 --latency-point off > $D/prof.log 2>&1
rc=$?
tail -n 3 $D/prof.log
find $D/prof -name "*kernel_stats.csv" | head
exit $rc

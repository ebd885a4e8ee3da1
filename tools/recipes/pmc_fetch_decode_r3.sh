set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r3j}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 32 --warmup 4 --latency-point off > $D/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D/pmc1 -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --latency-point off > $D/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D/pmc2 -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --lanes 2 --micro-batch 128 --latency-point off > $D/pmc2.log 2>&1
rc=$?
ls $D/prof $D/pmc1 $D/pmc2
exit $rc

# Round-3 (session 2) evidence run: kernel trace of the default W8A8 bench and of the bf16 bench,
# plus FETCH_SIZE of the bf16 1 x 256 decode GEMMs (weights read once per step).
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r3g}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 32 --warmup 4 --latency-point off > $D/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D/pmc_bf16 -o run --output-format csv -- python3 bench.py --quant none --steps 8 --warmup 2 --latency-point off > $D/pmc_bf16.log 2>&1
rc=$?
ls $D/prof $D/pmc_bf16
exit $rc

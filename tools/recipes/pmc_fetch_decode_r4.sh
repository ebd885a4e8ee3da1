# FETCH_SIZE per decode kernel for the round-4 default (2 lanes x 256 rows): one --pmc pass, then
# tools/pmc_fetch_summary.py with 64 dispatches per step (32 layers x 2 lanes)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r4t}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $D/pmc -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --latency-point off > $D/pmc.log 2>&1 || exit $?
python3 tools/pmc_fetch_summary.py $(find $D/pmc -name '*counter_collection.csv' | head -1) "FETCH_SIZE per decode kernel: bench.py default (2 lanes x 256), Llama-2-7B W8A8, 8 timed + 2 warm-up steps" 64 128 > $D/fetch.md || exit $?

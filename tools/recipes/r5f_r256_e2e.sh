# Round 5: packed qkv end to end — interleaved A/B on the headline config (r256_packed on / off),
# then the default bench's kernel table
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5f; mkdir -p $D
timeout -k 10 700 python3 tools/lane_ab.py --knobs "none;r256_packed=0" --reset "r256_packed=1" --lanes 2,1 --rounds 2 > $D/ab.jsonl 2> $D/ab.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/def -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/def.log 2>&1 || exit $?

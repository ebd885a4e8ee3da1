# Round-4: the headline config with an int8 KV cache (attention bytes halved) at 1 and 2 lanes of
# 256, plus the kernel table of the 1-lane run
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4v; mkdir -p $D
for L in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --lanes $L --kv-dtype int8 --latency-point off > $D/kv8_lanes$L.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --lanes 1 --kv-dtype int8 --latency-point off > $D/prof.log 2>&1 || exit $?

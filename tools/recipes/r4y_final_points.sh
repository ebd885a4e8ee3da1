# Round-4 final tree: default bench at 20 timed steps, and the reference's batch-1 configs (bf16 vs W8A8)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4yf; mkdir -p $D
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $D/bench20.log 2>&1 || exit $?
timeout -k 10 700 python3 tools/bench_reference_config.py --models llama-3.2-1b,pythia-1b,phi-2 --modes none,w8a8_smoothquant --repeats 3 > $D/refcfg.log 2>&1 || exit $?

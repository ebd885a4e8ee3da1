# the reference's batch-1 configs (tools/bench_reference_config.py) with the final round-5 tree:
# each model in its own precision (fp16 Phi-2 / Pythia, bf16 Llama-3.2-1B) and W8A8
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zl; mkdir -p $D
timeout -k 10 500 python3 tools/bench_reference_config.py --modes none,w8a8_smoothquant --repeats 2 > $D/ref.jsonl 2> $D/ref.err || exit $?

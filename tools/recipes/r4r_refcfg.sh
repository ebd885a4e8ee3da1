# Round-4: the reference's batch-1 points (Phi-2 / Pythia-1B / Llama-3.2-1B x bf16 / LLM.int8 / W8A8)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4refcfg; mkdir -p $D
timeout -k 10 900 python3 tools/bench_reference_config.py --repeats 3 > $D/refcfg.log 2>&1 || exit $?

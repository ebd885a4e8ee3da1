# Round 6: LLM.int8 gate_up with the SwiGLU in the one-launch GEMV's epilogue — tests, then the
# Llama-3.2-1B LLM.int8 batch-1 config (3 runs)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6ao; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -k "llmint8 or llm_int8" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python3 tools/bench_reference_config.py --models llama-3.2-1b --modes llm_int8 --repeats 2 > $D/ref_$i.jsonl 2> $D/ref_$i.err || { tail -20 $D/ref_$i.err; exit 1; }
  cut -c1-200 $D/ref_$i.jsonl
done

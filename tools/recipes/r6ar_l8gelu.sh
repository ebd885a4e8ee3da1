# Round 6: LLM.int8 up projection with the GELU in the one-launch GEMV's epilogue — tests, then
# the LLM.int8 batch-1 reference configs (2 runs)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6ar; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -k "llmint8 or llm_int8" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2; do
  timeout -k 10 400 python3 tools/bench_reference_config.py --modes llm_int8 --repeats 2 > $D/ref_$i.jsonl 2> $D/ref_$i.err || { tail -20 $D/ref_$i.err; exit 1; }
  python3 -c "
import json
for l in open('$D/ref_$i.jsonl'):
    d = json.loads(l); print('$i', d['model'], d['mode'], d['tps_incl_prompt'], d['p50_step_ms'])"
done

# Round 6: batch-1 LLM.int8 with the norms inside the one-launch projections
# LLM.int8 batch-1 configs with ONE_LAUNCH on (this tree) vs ab_old/ (three launches)
set -o pipefail
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r6ak; mkdir -p $D
cd $R
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_fp16_gpu.py -k "llmint8 or llm_int8 or norm or ln" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cd $R/ab_old; else cd $R; fi
    timeout -k 10 500 python3 tools/bench_reference_config.py --modes llm_int8 --repeats 2 > $D/ref_${v}_$i.jsonl 2> $D/ref_${v}_$i.err || { tail -20 $D/ref_${v}_$i.err; exit 1; }
    python3 -c "
import json
for l in open('$D/ref_${v}_$i.jsonl'):
    d = json.loads(l); print('$v $i', d['model'], d['mode'], d['tps_incl_prompt'], d['p50_step_ms'])"
  done
done

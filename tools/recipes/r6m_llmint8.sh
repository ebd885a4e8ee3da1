# Round 6: LLM.int8 at any rows on the device (no host sync): tests and the A/B against the
# round-5 host-sync form
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6m; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -k "llmint8" tests/test_fp16_gpu.py -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -3 $D/tests.log
timeout -k 10 300 python3 tools/llmint8_rows_ab.py > $D/ab.jsonl 2> $D/ab.err || { tail -20 $D/ab.err; exit 1; }
cat $D/ab.jsonl

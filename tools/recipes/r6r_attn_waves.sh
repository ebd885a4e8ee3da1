# Round 6: batch-1 decode attention with 4 / 8 / 16 waves per workgroup (same build, alternating)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6r; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -k "decode_attention_fused_b1_waves" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for i in 1 2; do
  for w in 4 8 16; do
    EDGELLM_TUNE="decode_attn_b1_waves=$w" timeout -k 10 300 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b_w${w}_$i.log 2>&1 || { tail -20 $D/b_w${w}_$i.log; exit 1; }
    echo "waves=$w $i $(grep '^{' $D/b_w${w}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done

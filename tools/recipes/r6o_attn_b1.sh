# Round 6: batch-1 decode attention, barrier-free double-buffered form with the first two K/V
# chunks issued at entry (default) vs the append-then-barrier form (decode_attn_early=0), same
# build, alternating; plus the decode-attention tests
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6o; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py -k "decode_attn or attention" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for i in 1 2 3; do
  for e in 0 1; do
    EDGELLM_TUNE="decode_attn_early=$e" timeout -k 10 300 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b_e${e}_$i.log 2>&1 || { tail -20 $D/b_e${e}_$i.log; exit 1; }
    echo "early=$e $i $(grep '^{' $D/b_e${e}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done

# Round-4: small MHA decode grids — double-buffered 4-wave form (0, default) vs single-buffered
# 16-wave form (1): tests, kernel A/B, batch-1 end to end
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4s16; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "small_grid or decode_attention_fused" > $D/tests.log 2>&1 || exit $?
for F in 0 1; do
  EDGELLM_TUNE="decode_attn_small=64,$F" timeout -k 10 300 python3 tools/attn_bench.py --shapes 1x200,1x512,1x1000 --only bf16 > $D/attn_f$F.log 2>&1 || exit $?
done
for F in 0 1; do
  EDGELLM_TUNE="decode_attn_small=64,$F" timeout -k 10 400 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b1_f$F.log 2>&1 || exit $?
done

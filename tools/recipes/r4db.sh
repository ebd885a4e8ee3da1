# Round-4: barrier-free double-buffered decode attention for small grids (decode_attn_small form 1)
# against the default routing (form 0): tests, kernel A/B (MHA 7B, GQA 1B shapes), batch-1 points
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4db; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "small_grid" > $D/tests.log 2>&1 || exit $?
for F in 0 1; do
  EDGELLM_TUNE="decode_attn_small=64,$F" timeout -k 10 300 python3 tools/attn_bench.py --shapes 1x200,1x512 --only bf16 > $D/attn7b_f$F.log 2>&1 || exit $?
  EDGELLM_TUNE="decode_attn_small=64,$F" timeout -k 10 300 python3 tools/attn_bench.py --shapes 1x264,1x700 --heads 32x8 --D 64 --only bf16 > $D/attn1b_f$F.log 2>&1 || exit $?
done
for F in 0 1; do
  EDGELLM_TUNE="decode_attn_small=64,$F" timeout -k 10 400 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b1_f$F.log 2>&1 || exit $?
  EDGELLM_TUNE="decode_attn_small=64,$F" timeout -k 10 600 python3 tools/bench_reference_config.py --models llama-3.2-1b --modes w8a8_smoothquant --repeats 3 > $D/ref1b_f$F.log 2>&1 || exit $?
done

# Round-4: batch-1 decode attention forms — barrier-free single-buffered (occ 4, default) vs the
# double-buffered form (occ 0): kernel A/B at batch-1 shapes and the end-to-end batch-1 points
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4occ; mkdir -p $D
for O in 4 0 5; do
  EDGELLM_TUNE="decode_attn_occ=$O" timeout -k 10 300 python3 tools/attn_bench.py --shapes 1x200,1x512,1x2048,16x200 --only bf16 > $D/attn_occ$O.log 2>&1 || exit $?
done
for O in 4 0; do
  EDGELLM_TUNE="decode_attn_occ=$O" timeout -k 10 400 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 --latency-point off > $D/b1_occ$O.log 2>&1 || exit $?
done

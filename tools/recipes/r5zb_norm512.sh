# 256-row decode: 512-thread norm over split-K slices (numerics, then alternating bench A/B on one box)
# (ran on the A/B build with tune key norm_part512; the 512-thread form was removed after this measurement)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5zb; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_rows256_gpu.py tests/test_fused_gpu.py -k "norm" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
for r in 1 2; do
for v in 1 0; do
  EDGELLM_TUNE="norm_part512=$v" timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/bench_n512_${v}_$r.log 2>&1 || exit $?
done
done

# Round-4: decode bookkeeping fused into the sampler's last launch (ops.sample_advance) — tests,
# then batch-1 A/B (EDGELLM_FUSE_ADVANCE=1 fused, 0 = sample + decode_advance), interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4sa; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_cogen_gpu.py tests/test_model_gpu.py tests/test_pipeline_gpu.py > $D/tests.log 2>&1 || exit $?
for F in 1 0 1 0; do
  EDGELLM_FUSE_ADVANCE=$F timeout -k 10 400 python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 8 \
    --latency-point off > $D/b1_fuse$F.$RANDOM.log 2>&1 || exit $?
done
for F in 1 0; do
  EDGELLM_FUSE_ADVANCE=$F timeout -k 10 500 python3 tools/bench_reference_config.py --models llama-3.2-1b \
    --modes none,w8a8_smoothquant --repeats 3 > $D/refcfg_fuse$F.log 2>&1 || exit $?
done

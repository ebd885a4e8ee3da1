# Round-4: batch-1 qkv GEMV with the attention tail — tests, bench latency point and the
# reference's 1B configs with the tail on / off (EDGELLM_ATT_TAIL_MAX=0)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4t; mkdir -p $D
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_att_tail_gpu.py \
  tests/test_fused_gpu.py -k "att_tail or gemv_norm or defers" > $D/tests.log 2>&1 || exit $?
for T in 1024 0; do
  EDGELLM_ATT_TAIL_MAX=$T timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $D/bench_tail$T.log 2>&1 || exit $?
  EDGELLM_ATT_TAIL_MAX=$T timeout -k 10 400 python3 tools/bench_reference_config.py --models llama-3.2-1b \
    --modes none,w8a8_smoothquant --repeats 2 > $D/ref1b_tail$T.log 2>&1 || exit $?
done

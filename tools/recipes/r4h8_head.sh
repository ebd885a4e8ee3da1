# Round-4: int8 LM head (tied heads included) — tests, the reference's batch-1 configs with it
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4h8; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k int8_lm_head > $D/tests.log 2>&1 || exit $?
timeout -k 10 900 python3 tools/bench_reference_config.py --modes none,w8a8_smoothquant --lm-head int8 --repeats 3 > $D/refcfg.log 2>&1 || exit $?

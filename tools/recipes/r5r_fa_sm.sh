# flash prefill: static priority for waves 4-7 and the deferred-max threshold (numerics, then A/B)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5r; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill_attention_fa" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/fa_ab.py --knob sm --rounds 6 --out $D/fa_sm_ab.json > $D/fa_ab.log 2>&1 || exit $?

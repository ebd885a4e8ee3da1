# flash prefill: scalar-base DMA addressing (numerics, interleaved A/B)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5x; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k "prefill" -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/fa_ab.py --knob saddr --rounds 8 --out $D/fa_saddr_ab.json > $D/fa_ab.log 2>&1 || exit $?

set -o pipefail
mkdir -p gpurun_out/r2k
timeout -k 10 400 python -u -m pytest tests/test_decode_numerics_gpu.py tests/test_model_gpu.py tests/test_fused_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r2k/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAIL|passed|failed|rel" gpurun_out/r2k/pytest.log | tail -15

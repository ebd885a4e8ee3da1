# Round 5: decode-step logits vs the fp32 reference at 200 rows, packed-activation qkv on / off
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5l; mkdir -p $D
EDGELLM_TUNE="r256_packed=0" timeout -k 10 300 python -u -m pytest tests/test_decode_numerics_gpu.py -q --timeout 200 --timeout-method thread -k "w8a8" > $D/off.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_decode_numerics_gpu.py -q --timeout 200 --timeout-method thread -k "w8a8" > $D/on.log 2>&1
exit 0

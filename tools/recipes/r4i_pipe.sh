# pipeline GPU tests: synchronous host staging vs side-stream pinned staging
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4i; mkdir -p $D
EDGELLM_PP_STAGE_SYNC=1 timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py > $D/sync.log 2>&1
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py -k "False-none-1-2" > $D/async.log 2>&1
EDGELLM_PP_STAGE_SYNC=1 timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_rccl_gpu.py > $D/rccl.log 2>&1
exit 0

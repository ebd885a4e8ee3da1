set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6j; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_b1_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -5 $D/tests.log
exit $rc

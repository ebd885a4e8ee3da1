set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6j; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_b1_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "1b" > $D/tests.log 2>&1; rc=$?
grep -E "h2 bad|e_h2|passed|failed" $D/tests.log | tail -8
exit $rc

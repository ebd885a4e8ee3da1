# Round 5: packed-activation 256-row kernel — exactness tests, then the lab A/B
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5e; mkdir -p $D
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_rows256_gpu.py > $D/pytest.log 2>&1 || exit $?
timeout -k 10 300 ./tools/.bin/r256_lab > $D/lab.jsonl 2> $D/lab.err || exit $?

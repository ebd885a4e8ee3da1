set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r3d}
mkdir -p $D
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rows256_gpu.py tests/test_fused_gpu.py tests/test_decode_numerics_gpu.py > $D/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_ops.py --only r256diag --out $D/diag.json > $D/diag.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --lanes 1 --micro-batch 256 --latency-point off > $D/bench_1x256.log 2>&1 && \
EDGELLM_DEC256_SCALES=token timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --lanes 1 --micro-batch 256 --latency-point off > $D/bench_1x256_tok.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --latency-point off > $D/bench_2x128.log 2>&1
rc=$?
tail -n 4 $D/*.log
exit $rc

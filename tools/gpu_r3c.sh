set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r3c}
mkdir -p $D
timeout -k 10 300 python -u tools/bench_ops.py --only r256diag --out $D/diag.json > $D/diag.log 2>&1
rc=$?
tail -n 5 $D/*.log
exit $rc

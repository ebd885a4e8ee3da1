set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/${1:-r3f}
mkdir -p $D
timeout -k 10 300 python -u tools/intmm_probe.py 256 > $D/intmm.log 2>&1
rc=$?
cat $D/intmm.log
exit $rc

# Round-4: multi-process CLI rehearsal tests on one GPU, lane-priority and 3-lane A/B
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4m; mkdir -p $D
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_multiproc_gpu.py > $D/multiproc.log 2>&1
for P in 0 1; do
  EDGELLM_LANE_PRIO=$P timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/prio$P.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --lanes 3 --latency-point off > $D/lanes3.log 2>&1 || exit $?

# Round-4: lane phase offset A/B (2 x 256 lanes; lane 1 starts OFFSET us after lane 0)
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4o; mkdir -p $D
for O in 0 60 110 170 0; do
  EDGELLM_LANE_OFFSET_US=$O timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-point off > $D/off$O.log 2>&1 || exit $?
  mv $D/off$O.log $D/off${O}_$(date +%s).log
done

set -o pipefail
mkdir -p gpurun_out/r2j
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2j/prof8 -o b1 -- python3 bench.py --micro-batch 1 --lanes 1 --steps 64 --warmup 4 --latency-point off > gpurun_out/r2j/prof8.log 2>&1; echo prof8 rc=$?; grep metric gpurun_out/r2j/prof8.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2j/prof16 -o b1 -- python3 bench.py --quant none --micro-batch 1 --lanes 1 --steps 64 --warmup 4 --latency-point off > gpurun_out/r2j/prof16.log 2>&1; echo prof16 rc=$?; grep metric gpurun_out/r2j/prof16.log | cut -c1-200
find gpurun_out/r2j -name "*kernel_trace*" -delete; find gpurun_out/r2j -name "*.db" -delete; du -sh gpurun_out/r2j

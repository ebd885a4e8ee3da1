set -o pipefail
mkdir -p gpurun_out/hi
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "headinfer or head_block or offload" > gpurun_out/hi/tests.log 2>&1 || { tail -30 gpurun_out/hi/tests.log; exit 1; }
tail -2 gpurun_out/hi/tests.log
timeout -k 10 240 python bench.py --model llama-3-8b --steps 32 --warmup 4 --headinfer-heads 4 > gpurun_out/hi/kernel.log 2>&1 || exit $?
tail -1 gpurun_out/hi/kernel.log | cut -c1-200; grep -o '"p50_token_latency_ms": [0-9.]*' gpurun_out/hi/kernel.log
EDGE_HEADINFER_COPY=dma timeout -k 10 240 python bench.py --model llama-3-8b --steps 32 --warmup 4 --headinfer-heads 4 > gpurun_out/hi/dma.log 2>&1 || exit $?
tail -1 gpurun_out/hi/dma.log | cut -c1-200
timeout -k 10 240 python bench.py --model llama-3-8b --steps 32 --warmup 4 --headinfer-heads 6 > gpurun_out/hi/kernel_h6.log 2>&1 || exit $?
tail -1 gpurun_out/hi/kernel_h6.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hi/prof -o hi -- python3 bench.py --model llama-3-8b --steps 16 --warmup 4 --headinfer-heads 4 > gpurun_out/hi/prof.log 2>&1; echo prof rc=$?

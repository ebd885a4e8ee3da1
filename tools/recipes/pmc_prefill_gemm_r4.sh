#!/bin/bash
# Prefill INT8 GEMM counters, qkv shape M=16384: the 128 x 256 16x16x64 kernel (x32 0) and the
# 256 x 256 32x32x32 kernel (x32 2), one PMC pass per rocprofv3 run, then tools/pmc_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r4p; mkdir -p $D
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE"
for x in 0 2; do
  timeout -k 10 120 python3 -u tools/pgemm_probe.py --x32 $x --intmm > $D/probe_$x.log 2>&1 || exit 1
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $P -d $D/x${x}_p$i -o run --output-format csv -- python3 tools/pgemm_probe.py --x32 $x --iters 10 > $D/x${x}_p$i.log 2>&1 || exit 1
  done
  python3 tools/pmc_summary.py "prefill GEMM qkv M=16384, x32=$x" $(find $D/x${x}_p1 $D/x${x}_p2 -name '*counter_collection.csv') > $D/pmc_x$x.md || exit 1
done
echo done

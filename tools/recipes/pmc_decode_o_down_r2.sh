#!/bin/bash
# Round 2 (ae): PMC counters for the 128-row o / down GEMVs (LDS-staged vs ring2).
set -o pipefail
mkdir -p gpurun_out/r2ae
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TA_BUSY_avr"
P3="FETCH_SIZE"
for sh in o down; do for r in 0 2; do
  for n in 1 2 3; do
    eval P=\$P$n
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/r2ae/${sh}_r${r}_p$n -- python3 tools/o_probe.py --shape $sh --ring $r --cfg 1 --iters 12 > gpurun_out/r2ae/${sh}_r${r}_p$n.log 2>&1 || { tail -5 gpurun_out/r2ae/${sh}_r${r}_p$n.log; exit 1; }
  done
done; done
echo done

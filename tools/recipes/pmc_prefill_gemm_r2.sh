#!/bin/bash
# Round 2 (n): prefill GEMM — hipBLASLt int8 reference point + PMC passes per form.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2n
for f in 2 3; do
  timeout -k 10 120 python -u tools/pgemm_probe.py --form $f --intmm > gpurun_out/r2n/probe_$f.log 2>&1 || exit 1
  grep TOPS gpurun_out/r2n/probe_$f.log
done
P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
Q="SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TA_BUSY_avr TA_TA_BUSY_sum"
for f in 2 3; do
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/r2n/pmc_a_$f -- python3 tools/pgemm_probe.py --form $f --iters 10 > gpurun_out/r2n/pmc_a_$f.log 2>&1 || { tail -5 gpurun_out/r2n/pmc_a_$f.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TA_BUSY_avr --kernel-trace --output-format csv -d gpurun_out/r2n/pmc_b_$f -- python3 tools/pgemm_probe.py --form $f --iters 10 > gpurun_out/r2n/pmc_b_$f.log 2>&1 || { tail -5 gpurun_out/r2n/pmc_b_$f.log; exit 1; }
done
echo done

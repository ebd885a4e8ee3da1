# Counter passes on the 256-row decode GEMMs (tools/r256_probe.py), one pass per rocprofv3 run.
#   bash tools/recipes/pmc_r256_r4.sh <outdir-tag> [probe args...]
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r4a}
shift || true
D=gpurun_out/$T
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P3="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $D/p$i -o run --output-format csv -- python3 tools/r256_probe.py "$@" > $D/p$i.log 2>&1 || exit $?
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/kt -o run --output-format csv -- python3 tools/r256_probe.py "$@" > $D/kt.log 2>&1 || exit $?
python3 tools/pmc_summary.py "256-row decode GEMM counters ($T)" $(find $D/p1 $D/p2 $D/p3 -name '*counter_collection.csv') > $D/pmc_summary.md
find $D/kt -name '*kernel_stats.csv' -exec cp {} $D/kernel_stats.csv \;
ls -R $D | head -40

# Counter passes on the decode attention kernels at the bench shape (256 x 170, Llama-2-7B heads):
# bf16 KV vs int8 KV (tools/attn_bench.py), one pass per rocprofv3 run, then the kernel trace
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-r4y}
D=gpurun_out/$T
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P3="TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $D/p$i -o run --output-format csv -- python3 tools/attn_bench.py --shapes 256x170 --only bf16,int8 > $D/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py "decode attention counters, 256 x 170 ($T)" --min-calls 4 $(find $D/p1 $D/p2 $D/p3 -name '*counter_collection.csv') > $D/pmc_summary.md

# Round 6: counters of the SHIPPED decode kernels at the bench shape (bench.py one lane x 256 rows,
# Llama-2-7B W8A8), one rocprofv3 pass each, + the list of counters this box offers
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6e; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $D/counters_list.txt 2>&1 || true
B="bench.py --lanes 1 --steps 6 --warmup 2 --latency-point off --prompt-len 128"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
P2="TA_BUSY_avr TA_TA_BUSY_sum FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $P -d $D/p$i -o run --output-format csv -- python3 $B > $D/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py "shipped decode kernels, bench.py 1 x 256 (r6)" --min-calls 100 $(find $D/p1 $D/p2 -name '*counter_collection.csv') > $D/pmc_summary.md
# keep the summary, drop the raw per-dispatch CSVs (gpurun merges back at most 64 MiB)
rm -rf $D/p1 $D/p2

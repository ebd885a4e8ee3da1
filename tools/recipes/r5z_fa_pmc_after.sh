# (after the asm transposed V reads) counter passes on fa_kernel at the 32K causal shape (Llama-3-8B heads), one pass per rocprofv3 run
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5z
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $D/p$i -o run --output-format csv -- python3 tools/fa_probe.py --calls 3 > $D/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py "fa_kernel counters, 32K causal, Hq 32 / Hkv 8, D 128" --min-calls 2 $(find $D/p1 $D/p2 -name '*counter_collection.csv') > $D/pmc_summary.md
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/prefill_profile.py --model llama-3-8b --prompt-len 32768 --reps 1 > $GRAFT_REPO_ROOT/$D/ttft.log 2>&1 || exit $?

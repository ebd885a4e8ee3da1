# Round 6: Table-3-style ensemble runs on the current tree (tools/ensemble_table3.sh), logs under gpurun_out/ens
set -o pipefail
export PYTHONUNBUFFERED=1
T=300 N=64 bash tools/ensemble_table3.sh 2>&1 | tee gpurun_out/ens_summary.txt

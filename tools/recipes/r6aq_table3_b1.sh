# Round 6 (final tree: + the LLM.int8 SwiGLU epilogue): the batch-1 Table-3 combo rows again
set -o pipefail
mkdir -p gpurun_out/ens_r6e
N=${N:-64}
python3 - <<PY
import csv, os
src = "llm-for-distributed-egde-devices_amd/data/nq_sample.csv"
rows = list(csv.DictReader(open(src)))
with open("gpurun_out/ens_r6e/nq_rep.csv", "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=["query", "answer"])
    w.writeheader()
    for i in range(1000):
        w.writerow(rows[i % len(rows)])
PY
C="python3 -m edgellm.cli.combine"
D="--dataset_path gpurun_out/ens_r6e/nq_rep.csv"
run() { name=$1; shift; timeout -k 10 ${T:-500} "$@" > gpurun_out/ens_r6e/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -E "Tokens/Sec|Time Taken|Memory|Agg" gpurun_out/ens_r6e/$name.log | tail -4; [ $rc -eq 0 ] || exit $rc; }
run combo_base_b1      $C --config configs/ensemble.yaml $D --num_samples 16
run combo_llmint8_b1   $C --config configs/ensemble_int8.yaml $D --num_samples 12
run combo_w8a8_b1      $C --config configs/ensemble.yaml $D --num_samples 16 --quant w8a8_smoothquant

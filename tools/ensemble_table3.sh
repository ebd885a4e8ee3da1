# Table-3-style ensemble efficiency runs on one MI355X (random-init weights of the reference's
# architectures; the bundled NQ sample rows repeated to N questions).  Writes gpurun_out/ens/*.log
set -o pipefail
mkdir -p gpurun_out/ens
N=${N:-64}
python3 - <<PY
import csv, os
src = "llm-for-distributed-egde-devices_amd/data/nq_sample.csv"
rows = list(csv.DictReader(open(src)))
with open("gpurun_out/ens/nq_rep.csv", "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=["query", "answer"])
    w.writeheader()
    for i in range(1000):
        w.writerow(rows[i % len(rows)])
PY
C="python3 -m edgellm.cli.combine"
D="--dataset_path gpurun_out/ens/nq_rep.csv"
run() { name=$1; shift; timeout -k 10 ${T:-500} "$@" > gpurun_out/ens/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -E "Tokens/Sec|Time Taken|Memory|Agg" gpurun_out/ens/$name.log | tail -4; [ $rc -eq 0 ] || exit $rc; }
run combo_base_b1      $C --config configs/ensemble.yaml $D --num_samples 16
run combo_base_b16     $C --config configs/ensemble.yaml $D --num_samples 64 --batch_size 16
run combo_llmint8_b1   $C --config configs/ensemble_int8.yaml $D --num_samples 12
run combo_w8a8_b1      $C --config configs/ensemble.yaml $D --num_samples 16 --quant w8a8_smoothquant
run combo_w8a8_b16     $C --config configs/ensemble.yaml $D --num_samples 64 --batch_size 16 --quant w8a8_smoothquant
run north_star_vote    $C --config configs/north_star.yaml $D --num_samples 32 --batch_size 16
# agents sharing the GPU decode side by side on their own streams (orchestrator run_agents ->
# engine co_generate), 128 questions per batch
run north_star_vote_b256 $C --config configs/north_star.yaml $D --num_samples 512 --batch_size 256 --max_seq 512
run combo_base_b128    $C --config configs/ensemble.yaml $D --num_samples 256 --batch_size 128
run combo_w8a8_b128    $C --config configs/ensemble.yaml $D --num_samples 256 --batch_size 128 --quant w8a8_smoothquant

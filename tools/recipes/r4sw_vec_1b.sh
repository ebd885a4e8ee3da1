# Round-4: Llama-3.2-1B batch-1 (128K vocab) with and without the 16-byte sampler chunk loads, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r4sw; mkdir -p $D
for N in 1 0 1 0; do
  EDGELLM_TUNE="sample_vec=$N" timeout -k 10 400 python3 tools/bench_reference_config.py --models llama-3.2-1b \
    --modes none,w8a8_smoothquant --repeats 3 > $D/refcfg_v$N.$RANDOM.log 2>&1 || exit $?
done

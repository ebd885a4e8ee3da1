# Round 5: fp16 kernel instantiations (norm / rope / decode + prefill attention / GEMV) against the
# fp32 reference, the existing kernel + model suites, then the reference's batch-1 points in the
# reference's own precision (fp16 Phi-2 / Pythia, bf16 Llama-3.2-1B) and bf16 for comparison
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r5g; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_fp16_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/bench_reference_config.py --modes none --repeats 2 > $D/ref_fp.jsonl 2> $D/ref_fp.err || exit $?
timeout -k 10 400 python3 tools/bench_reference_config.py --models phi-2,pythia-1b --modes none --precision bf16 --repeats 2 > $D/ref_bf16.jsonl 2> $D/ref_bf16.err || exit $?

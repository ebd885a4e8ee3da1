#!/bin/bash
# Round 2 (ad): full GPU suite after the packed-A prefill default.
set -o pipefail
mkdir -p gpurun_out/r2ad
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ad/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r2ad/pytest.log
exit $rc

#!/bin/bash
# Round 2 (v): L2 -> CU ingest ceiling (VGPR loads vs LDS-DMA), no MFMA.
set -o pipefail
mkdir -p gpurun_out/r2v /tmp/ib
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/ingest_bw.hip -o /tmp/ib/ingest_bw || exit 1
timeout -k 10 120 /tmp/ib/ingest_bw > gpurun_out/r2v/ingest.csv 2>&1; rc=$?; cat gpurun_out/r2v/ingest.csv; exit $rc

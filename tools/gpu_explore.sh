#!/bin/bash
# per-shape GEMM table (eager), C1 (CLIP-only) bench line, PMC traffic of the dominant GEMM
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gemm-table --no-cpu-baseline --no-parity --steps 5 > gpurun_out/table.json 2> gpurun_out/table.err || { tail -30 gpurun_out/table.err; exit 1; }
cat gpurun_out/table.json
timeout -k 10 300 python -u bench.py --mask-ratio 0 --no-cpu-baseline --no-parity > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail -30 gpurun_out/c1.err; exit 1; }
cat gpurun_out/c1.json
TAG=dom bash tools/pmc_traffic.sh 50432 2048 512 0 1 5

#!/bin/bash
# Kernel diagnostics: phase ablations + per-phase cycle breakdown.  Outputs under gpurun_out/.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/phase_timing.py fastq 10 > gpurun_out/phase.log 2>&1 || exit 1
DBGS="${DBGS:-0 1 2 3 4 32}" timeout -k 10 400 bash tools/ablate.sh 10 > gpurun_out/ablate.log 2>&1

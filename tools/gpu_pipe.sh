#!/bin/bash
# parity tests, then phase timing + A/B bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/phase_timing.py fastq 10 > gpurun_out/phase.log 2>&1 || exit 1
bash tools/gpu_ab.sh

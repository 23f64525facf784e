#!/bin/bash
# parity tests (stop at first failure) then an A/B timing pass
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
bash tools/gpu_ab.sh

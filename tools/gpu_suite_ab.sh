#!/bin/bash
# The whole -m gpu suite, then an interleaved A/B of libshockidx variants ($VARS, format $FMT).
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
VARS=${VARS:-base} ROUNDS=${ROUNDS:-3} FMT=${FMT:-fasta} bash tools/gpu_ab.sh || exit 1
exit 0

#!/bin/bash
# Iteration pass: GPU parity tests, k_pipe phase breakdown, bench (no CPU leg).  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
SHOCKIDX_VARIANT=diag timeout -k 10 200 python -u tools/phase_timing.py fastq 10 > $O/phase.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --cpu-sec 0 ${BENCH_ARGS} > $O/bench_iter.json 2> $O/bench_iter.err || exit 1
exit 0

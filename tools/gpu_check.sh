#!/bin/bash
# One GPU-box pass: parity tests, the bench, a rocprofv3 kernel-trace of the bench,
# a repeat-determinism check.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
nproc > gpurun_out/nproc.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sec 10 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-sec 0 > gpurun_out/bench_prof.log 2>&1 && \
timeout -k 10 300 python -u tools/repeat_check.py fastq 10 10 auto > gpurun_out/rep.log 2>&1

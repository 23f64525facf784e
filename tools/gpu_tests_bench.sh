#!/bin/bash
# GPU parity tests, then both bench lines (no CPU leg).  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for f in fastq fasta; do
  timeout -k 10 300 python -u bench.py --fmt $f --cpu-sec 0 > $O/bench_tb_$f.json 2> $O/bench_tb_$f.err || exit 1
done
exit 0

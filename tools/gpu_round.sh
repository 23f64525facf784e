#!/bin/bash
# Round measurement: GPU tests, FASTQ (C2) + FASTA (C3) bench lines with kernel traces and
# HBM PMC passes, the end-to-end host-memory rate.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
TAG=${TAG:-r01} FMT=fastq bash tools/gpu_measure.sh || exit 1
SKIP_TESTS=1 TAG=${TAG:-r01} FMT=fasta bash tools/gpu_measure.sh || exit 1
timeout -k 10 400 python -u bench.py --e2e --steps 3 --warmup 1 > $O/bench_e2e_fastq.json 2> $O/bench_e2e_fastq.err || exit 1

timeout -k 10 600 python -u bench.py --subset --steps 5 --warmup 2 > $O/bench_subset.json 2> $O/bench_subset.err || exit 1
exit 0

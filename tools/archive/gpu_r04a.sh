#!/bin/bash
# round-4 measurement batch: allocation probe, the -m gpu suite, bench lines + kernel traces,
# the fd end-to-end line, and an interleaved A/B of FASTQ tile-pass variants.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/placement_probe.py 4 > $O/placement3.txt 2>&1 || exit 1
cat $O/placement3.txt
FMTS="fastq fasta" bash tools/gpu_iter.sh || exit 1
timeout -k 10 300 python bench.py --kind line --cpu-sec 0 --steps 20 --warmup 3 > $O/it_bench_line.json 2> $O/it_bench_line.err || exit 1
head -c 700 $O/it_bench_line.json; echo
timeout -k 10 300 python bench.py --e2e --fd --steps 3 --warmup 1 > $O/e2e_fd.json 2> $O/e2e_fd.err || exit 1
head -c 900 $O/e2e_fd.json; echo
VARS="base nt1 w8" ROUNDS=3 FMT=fastq bash tools/gpu_ab.sh || exit 1
exit 0

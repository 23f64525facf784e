#!/bin/bash
# round-4 batch: the -m gpu suite, FASTQ / FASTA / line bench lines with kernel traces, the fd
# end-to-end line, an interleaved A/B of the FASTQ DMA policy (nt0 = default-policy body).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
FMTS="fastq fasta" bash tools/gpu_iter.sh || exit 1
rm -rf $O/it_kt_line
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/it_kt_line -o kt --output-format csv -- python3 bench.py --kind line --cpu-sec 0 --steps 20 --warmup 3 > $O/it_bench_line.json 2> $O/it_bench_line.err || exit 1
head -c 700 $O/it_bench_line.json; echo
VARS="base nt0" ROUNDS=3 FMT=fastq bash tools/gpu_ab.sh || exit 1
for c in "fastq fq2fa" "fastq anonymize"; do
  set -- $c
  rm -rf $O/filt_kt_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/filt_kt_$1_$2 -o run -- python3 bench.py --kind filter --fmt $1 --filter $2 --steps 5 --warmup 1 > $O/bench_filter_$1_$2.json 2> $O/bench_filter_$1_$2.err || exit 1
  head -c 600 $O/bench_filter_$1_$2.json; echo
done
exit 0

#!/bin/bash
# Round-3 check: the -m gpu suite, the three default bench lines, a kernel trace of the FASTQ
# bench (per-kernel times of the whole build).  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
for f in fastq fasta; do
  timeout -k 10 300 python -u bench.py --fmt $f --cpu-sec 0 > $O/bench_$f.json 2> $O/bench_$f.err || exit 1
done
timeout -k 10 300 python -u bench.py --kind line --cpu-sec 0 > $O/bench_line.json 2> $O/bench_line.err || exit 1
rm -rf $O/prof_kt_fastq
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_kt_fastq -o kt --output-format csv -- python3 $R/bench.py --fmt fastq --steps 20 --warmup 3 --cpu-sec 0 > $O/bench_kt_fastq.json 2> $O/bench_kt_fastq.err || exit 1
find $O/prof_kt_fastq -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_fastq.csv \;
exit 0

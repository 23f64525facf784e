#!/bin/bash
# round-end measurement: full GPU suite + FASTQ PMC/trace, FASTA PMC/trace, line bench + trace
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
TAG=${TAG:-r02} FMT=fastq bash tools/gpu_measure.sh || exit 1
echo "pytest: $(tail -1 $O/pytest_gpu.log)"
SKIP_TESTS=1 TAG=${TAG:-r02} FMT=fasta bash tools/gpu_measure.sh || exit 1
timeout -k 10 300 python -u bench.py --kind line --steps 20 --warmup 3 > $O/bench_line.json 2> $O/bench_line.err || exit 1
rm -rf $O/prof_kt_line
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_kt_line -o kt --output-format csv -- python3 bench.py --kind line --steps 20 --warmup 3 > $O/bench_kt_line.json 2> $O/bench_kt_line.err || exit 1
cat $O/bench_fastq.json $O/bench_fasta.json $O/bench_line.json

#!/bin/bash
# One measurement pass on the GPU box: parity tests, the bench line, a rocprofv3 kernel trace
# of the same bench command, and the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE: one block
# each, separate runs).  Everything lands under gpurun_out/; copy what is judged to profiles/.
#   TAG=r01 FMT=fastq bash tools/gpu_measure.sh
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out
TAG=${TAG:-r01}
FMT=${FMT:-fastq}
mkdir -p $O
nproc > $O/nproc.log
lscpu > $O/lscpu.log 2>&1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
fi
timeout -k 10 300 python -u bench.py --fmt $FMT > $O/bench_$FMT.json 2> $O/bench_$FMT.err || exit 1
rm -rf $O/prof_kt_$FMT $O/prof_fetch_$FMT $O/prof_write_$FMT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_kt_$FMT -o kt --output-format csv -- python3 $R/bench.py --fmt $FMT --steps 20 --warmup 3 --cpu-sec 0 > $O/bench_kt_$FMT.json 2> $O/bench_kt_$FMT.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_$FMT -o pmc --output-format csv -- python3 $R/bench.py --fmt $FMT --steps 3 --warmup 1 --cpu-sec 0 --no-check > $O/bench_fetch_$FMT.json 2> $O/bench_fetch_$FMT.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_$FMT -o pmc --output-format csv -- python3 $R/bench.py --fmt $FMT --steps 3 --warmup 1 --cpu-sec 0 --no-check > $O/bench_write_$FMT.json 2> $O/bench_write_$FMT.err || exit 1
python tools/pmc_summary.py $O/prof_kt_$FMT $O/prof_fetch_$FMT $O/prof_write_$FMT $O/pmc_${TAG}_$FMT.json $FMT > $O/pmc_${TAG}_$FMT.log 2>&1
exit 0

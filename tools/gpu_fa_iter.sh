#!/bin/bash
# FASTA iteration: GPU suite, FASTA bench line, kernel trace of the same command
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
for f in ${FMTS:-fasta}; do
  timeout -k 10 300 python -u bench.py --fmt $f --cpu-sec 0 > $O/bench_it_$f.json 2> $O/bench_it_$f.err || exit 1
  rm -rf $O/prof_it_$f
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_it_$f -o kt --output-format csv -- python3 bench.py --fmt $f --cpu-sec 0 > $O/bench_itkt_$f.json 2> $O/bench_itkt_$f.err || exit 1
  cat $O/bench_it_$f.json
done

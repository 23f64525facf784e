#!/bin/bash
# line index iteration: line GPU tests, the line bench line and its kernel trace
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "line" --timeout 120 --timeout-method thread > $O/pytest_line.log 2>&1 || { tail -30 $O/pytest_line.log; exit 1; }
tail -1 $O/pytest_line.log
rm -rf $O/prof_it_line
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_it_line -o kt --output-format csv -- python3 bench.py --kind line --steps 20 --warmup 3 > $O/bench_it_line.json 2> $O/bench_it_line.err || exit 1
grep -h "k_line" $O/prof_it_line/kt_kernel_stats.csv | cut -d, -f1-4

#!/bin/bash
# Subset / filter / chunkrecord / part GPU tests, the C4 subset bench line, the streaming
# microbenchmark.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_subset.py tests/test_gpu_filter.py tests/test_gpu_chunk.py tests/test_gpu_part.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_sub.log 2>&1 || { tail -30 $O/pytest_sub.log; exit 1; }
tail -2 $O/pytest_sub.log
timeout -k 10 600 python -u bench.py --subset --steps 5 --warmup 2 > $O/bench_subset.json 2> $O/bench_subset.err || { tail -5 $O/bench_subset.err; exit 1; }
cat $O/bench_subset.json
SB_SKEL=1 timeout -k 10 300 ./tools/streambench 10 10 > $O/streambench.txt 2>&1 || exit 1
cat $O/streambench.txt
exit 0

#!/bin/bash
# round 5: the FASTQ density-mix test (packed start arrays of every length), the C4 line traced
set -o pipefail
O=gpurun_out/r05q2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "density or generated or blank" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt_subset -o kt --output-format csv -- python3 bench.py --subset --steps 5 --warmup 2 > $O/bench_subset.json 2> $O/bench_subset.err || exit $?

#!/bin/bash
# round 5: subset index -- the id text's line ends by three small kernels (no line tile pass),
# oSize over 64 slots, one parent-row read per id; the subset suites, then the C4 line traced
set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_subset.py tests/test_gpu_chunk.py tests/test_gpu_part.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt_subset -o kt --output-format csv -- python3 bench.py --subset --steps 5 --warmup 2 > $O/bench_subset.json 2> $O/bench_subset.err || exit $?

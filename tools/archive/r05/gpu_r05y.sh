#!/bin/bash
# round 5: the small-input scan (three plain launches) against the single-pass look-back scan on
# the whole C4 subset node; then the subset / filter / chunkrecord suites (every caller of the scan)
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_subset.py tests/test_gpu_filter.py tests/test_gpu_chunk.py tests/test_gpu_part.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_subset.py base sc0 --rounds 6 --per 10 > $O/ab_subset.json 2> $O/ab_subset.err || exit $?

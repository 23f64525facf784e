#!/bin/bash
# round 5: the subset gather: two chunks per lane in flight (base) against one (gk0), 512 / 128 threads, 8 / 32 KiB blocks
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_subset.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_gather.py base gk0 gt512 gt128 gb8k gb32k --rounds 6 --per 10 > $O/ab_gather.json 2> $O/ab_gather.err || exit $?

#!/bin/bash
# round 5: the subset gather: 16 / 32 / 64 KiB output blocks per workgroup, 256 / 128 threads
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_subset.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_gather.py base gb32k gt128 gb32t128 gb64k gb64t128 --rounds 6 --per 10 > $O/ab_gather.json 2> $O/ab_gather.err || exit $?

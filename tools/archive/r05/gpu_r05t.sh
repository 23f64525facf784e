#!/bin/bash
# round 5: FASTQ suites after the k_fq_place staging fix; the placement / reallocation probe
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_integrity.py tests/test_gpu_filter.py tests/test_gpu_slabs.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/probes/placement_realloc.py > $O/placement_realloc.json 2> $O/placement_realloc.err || exit $?

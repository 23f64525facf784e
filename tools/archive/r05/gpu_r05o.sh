#!/bin/bash
# round 5: the LDS-staged subset gather against the round-4 gather (one process, the same runs),
# the FASTA tile pass with its pieces validated in the candidate loop against the separate loop,
# the gather / subset / FASTA suites on the default build
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_subset.py tests/test_gpu_fasta_tiles.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_gather.py base gl0 --rounds 6 --per 10 > $O/ab_gather.json 2> $O/ab_gather.err || exit $?
timeout -k 10 400 python -u tools/ab_inproc.py base fi0 --fmt fasta --copies 4 --rounds 4 --per 8 --warmup 8 > $O/ab_fa.json 2> $O/ab_fa.err || exit $?

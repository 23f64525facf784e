#!/bin/bash
# round 5: the FASTA tile certificate's lookup over two mask words (base) against the loop (tc0)
set -o pipefail
O=gpurun_out/r05fc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fasta_tiles.py tests/test_gpu_parity.py -k "fasta or generated or kat or fixture" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/ab_inproc.py base tc0 --fmt fasta --copies 4 --rounds 4 --per 5 --warmup 5 --turn-warmup 20 > $O/ab_fa.json 2> $O/ab_fa.err || exit $?

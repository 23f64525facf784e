#!/bin/bash
# round 5: FASTA fast path over two mask words (default now) -- FASTA suites; four words (fnl4) A/B
set -o pipefail
O=gpurun_out/r05fb
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fasta_tiles.py tests/test_gpu_parity.py tests/test_gpu_integrity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/ab_inproc.py base fnl4 --fmt fasta --copies 4 --rounds 4 --per 5 --warmup 5 --turn-warmup 20 > $O/ab_fa.json 2> $O/ab_fa.err || exit $?

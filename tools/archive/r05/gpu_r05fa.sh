#!/bin/bash
# round 5: FASTA piece check's fast path over two mask words (fnl2) against one (base)
set -o pipefail
O=gpurun_out/r05fa
mkdir -p $O
timeout -k 10 600 python -u tools/ab_inproc.py base fnl2 --fmt fasta --copies 4 --rounds 4 --per 5 --warmup 5 --turn-warmup 20 > $O/ab_fa.json 2> $O/ab_fa.err || exit $?

#!/bin/bash
# round 5: FASTA pieces validated in the candidate loop, entries stored by wave 0 after the last
# barrier (fin) against the separate validation loop (base); then the FASTA suites on fin's sources
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 600 python -u tools/ab_inproc.py base fin --fmt fasta --copies 4 --rounds 4 --per 5 --warmup 5 --turn-warmup 20 > $O/ab_fa.json 2> $O/ab_fa.err || exit $?

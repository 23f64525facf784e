#!/bin/bash
# round 5: tile order / store policy variants over 4 separately allocated copies of the input
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 400 python -u tools/ab_inproc.py base ring0 r0opq8 s1 s2 nt0s ntout --copies 4 --rounds 6 --per 10 > $O/ab_copies.json 2> $O/ab_copies.err || exit $?

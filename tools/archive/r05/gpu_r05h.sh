#!/bin/bash
# round 5: is the placement sensitivity in the row-start stores? (abl4: none; its tables are wrong)
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 400 python -u tools/ab_inproc.py ring0 abl4 r0nolean8 s2 --copies 4 --rounds 6 --per 10 > $O/ab_copies.json 2> $O/ab_copies.err || exit $?

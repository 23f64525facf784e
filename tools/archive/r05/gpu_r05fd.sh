#!/bin/bash
# round 5: FASTQ plus-line ID compare, 32 bytes per LDS round (idc) against 16 (base)
set -o pipefail
O=gpurun_out/r05fd
mkdir -p $O
timeout -k 10 600 python -u tools/ab_inproc.py base idc --copies 4 --rounds 4 --per 5 --warmup 5 --turn-warmup 20 > $O/ab_fq.json 2> $O/ab_fq.err || exit $?

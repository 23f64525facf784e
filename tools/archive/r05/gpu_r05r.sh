#!/bin/bash
# round 5: FASTQ start-array layouts over 6 input copies: packed + the workgroups' streams
# interleaved line by line (base), packed (il0), round 4's padded regions (pk0), padded regions
# 32 KiB apart (sk256), no row-start stores (abl4)
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 600 python -u tools/ab_inproc.py base il0 pk0 sk256 abl4 --copies 6 --rounds 3 --per 5 --warmup 5 > $O/ab_fq.json 2> $O/ab_fq.err || exit $?

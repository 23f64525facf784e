#!/bin/bash
# round 5: does the FASTQ tile pass's store penalty scale with the bytes stored?  The same kernel
# flushing 1/2, 1/4, 1/8 of its ring lines (timing only: tables wrong), 20 untimed builds per turn
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 900 python -u tools/ab_inproc.py base pk0 half quarter eighth --copies 4 --rounds 4 --per 5 --warmup 5 --turn-warmup 20 > $O/ab_fq.json 2> $O/ab_fq.err || exit $?

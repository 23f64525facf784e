#!/bin/bash
# round 5: FASTQ stage regions padded and their starts skewed (does the placement penalty follow
# where the writes land relative to the read stream?) over 6 input copies; the gather with /
# without the skipped words
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python -u tools/ab_inproc.py base sk37 sk1 sk256 sk101 abl4 --copies 6 --rounds 3 --per 5 --warmup 5 > $O/ab_fq.json 2> $O/ab_fq.err || exit $?
timeout -k 10 300 python -u tools/ab_gather.py base gs0 gk0 --rounds 6 --per 10 > $O/ab_gather.json 2> $O/ab_gather.err || exit $?

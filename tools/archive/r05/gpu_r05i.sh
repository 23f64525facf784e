#!/bin/bash
# round 5: where the FASTQ row starts go (fixed slots / per-workgroup regions NT or cached /
# per-XCD append logs) over 4 separately allocated copies of the input
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 400 python -u tools/ab_inproc.py ring0 base ringT xlog xlogopq8 abl4 --copies 4 --rounds 6 --per 10 > $O/ab_copies.json 2> $O/ab_copies.err || exit $?

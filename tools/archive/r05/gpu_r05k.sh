#!/bin/bash
# round 5: where the row-start stores cost (burst flushes; stores into 8 hot slots, cached / nt;
# cached fixed slots) over 6 input copies
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 600 python -u tools/ab_inproc.py ring0 rb1k rb2k sinkT sinkNT r0T base --copies 6 --rounds 3 --per 6 --warmup 6 > $O/ab_copies.json 2> $O/ab_copies.err || exit $?

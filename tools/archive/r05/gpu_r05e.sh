#!/bin/bash
# round 5: in-process paired A/B of the FASTQ tile-pass variants (tools/ab_inproc.py)
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 python -u tools/ab_inproc.py base ring0 lean0 r0lean r0lean8 r0opq r0opq8 t8k --rounds 16 --per 10 > $O/ab_inproc_1.json 2> $O/ab_inproc_1.err || exit $?
timeout -k 10 300 python -u tools/ab_inproc.py base ring0 lean0 r0lean r0lean8 r0opq r0opq8 t8k --rounds 16 --per 10 > $O/ab_inproc_2.json 2> $O/ab_inproc_2.err || exit $?

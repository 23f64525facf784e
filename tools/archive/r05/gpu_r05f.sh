#!/bin/bash
# round 5: does the input's placement set the FASTQ build's speed (tools/ab_placement.py), twice
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 300 python -u tools/ab_placement.py > $O/placement_1.json 2> $O/placement_1.err || exit $?
timeout -k 10 300 python -u tools/ab_placement.py --copies plain,contig,plain,contig,plain,contig --rounds 4 > $O/placement_2.json 2> $O/placement_2.err || exit $?

#!/bin/bash
# round 5: denser fixed row-start slots (256 / 128 B per tile instead of 1 KiB) over 4 input
# copies; then the drop-in create with and without the shim's trim between builds
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 170 python -u tools/ab_inproc.py ring0 r0s128 r0s64 base --copies 4 --rounds 5 --per 10 > $O/ab_copies.json 2> $O/ab_copies.err || exit $?
timeout -k 10 170 python bench.py --e2e --fd --steps 6 --warmup 1 > $O/e2e_fd_keep.json 2> $O/e2e_fd_keep.err || exit $?
timeout -k 10 170 python bench.py --e2e --fd --steps 6 --warmup 1 --trim 1 > $O/e2e_fd_trim1.json 2> $O/e2e_fd_trim1.err || exit $?

#!/bin/bash
# Same-box floor comparison: the streaming microbenchmark's skeletons, then k_fq_tiles as built
# (base), without certification (abl1) and with the staging alone (abl3).
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
SB_SKEL=1 timeout -k 10 300 ./tools/streambench 10 10 > $O/streambench.txt 2>&1 || exit 1
cat $O/streambench.txt
SHOCKIDX_DEBUG=1 VARS="${VARS:-base abl1 abl3}" ROUNDS=${ROUNDS:-2} FMT=fastq bash tools/gpu_ab.sh || exit 1
exit 0

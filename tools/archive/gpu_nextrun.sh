#!/bin/bash
# chunkrecord k_cr_next_fq: runs of 4 records per thread walking forward (base) vs one record per
# thread (nrun1) vs runs of 8 (nrun8) -- chunkrecord GPU tests, then A/B of the FASTQ build.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chunk.py -x -q --timeout 300 --timeout-method thread > $O/nextrun_tests.log 2>&1 || { tail -30 $O/nextrun_tests.log; exit 1; }
tail -1 $O/nextrun_tests.log
KIND=chunkrecord VARS="base nrun1 nrun8" ROUNDS=2 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_cr_next_run.txt
exit 0

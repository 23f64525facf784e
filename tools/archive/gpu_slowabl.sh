#!/bin/bash
# Where k_fq_tiles spends its time fresh and in the slow state after sustained load: the kernel
# against its ablations (ablT1 no record validation, ablT2 no positions either, ablT3 no masks
# either = the staging alone), interleaved, before and after the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
VARS="base ablT1 ablT2 ablT3" ROUNDS=2 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_slowabl_fresh.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/slowabl_suite.log 2>&1 || exit 1
VARS="base ablT1 ablT2 ablT3" ROUNDS=2 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_slowabl_after.txt
exit 0

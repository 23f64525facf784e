#!/bin/bash
# The tile passes' stores fresh and in the slow state after sustained load: FASTQ without its
# row-start stores (ablT4) and the line pass without its position stores (ablL1), interleaved
# with the kernels as built, before and after the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
ab() {
  VARS="base ablT4" ROUNDS=2 bash tools/gpu_ab.sh || return 1
  cp $O/ab_fastq.txt $O/ab_stores_fastq_$1.txt
  KIND=line VARS="base ablL1" ROUNDS=2 bash tools/gpu_ab.sh || return 1
  cp $O/ab_fastq.txt $O/ab_stores_line_$1.txt
}
ab fresh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/slowabl2_suite.log 2>&1 || exit 1
ab after || exit 1
cat $O/ab_stores_*_fresh.txt $O/ab_stores_*_after.txt
exit 0

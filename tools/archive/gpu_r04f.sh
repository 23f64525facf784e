#!/bin/bash
# Round 4, late: the FASTQ writer's chunk -> record map -- the filter GPU tests, then A/B against
# the binary search per chunk (fwbs), anonymize and fq2fa; FASTA anonymize with its writer's
# next-step load issued early vs not (fapre0).
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_filter.py -x -q --timeout 300 --timeout-method thread > $O/r04f_tests.log 2>&1 || { tail -30 $O/r04f_tests.log; exit 1; }
tail -2 $O/r04f_tests.log
KIND=filter FILTER=anonymize VARS="base fwbs" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_fw_anonymize.txt
KIND=filter FILTER=fq2fa VARS="base fwbs" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_fw_fq2fa.txt
FMT=fasta KIND=filter FILTER=anonymize VARS="base fapre0" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fasta.txt $O/ab_fa_anon_prefetch.txt
exit 0

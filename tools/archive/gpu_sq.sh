#!/bin/bash
# SQ counters (two passes each) of the FASTQ and FASTA tile kernels; outputs gpurun_out/sq_<fmt>_<i>/.
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
i=0
for fmt in fastq fasta; do
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES"; do
  i=$((i+1)); rm -rf $O/sq_${fmt}_$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/sq_${fmt}_$i -o pmc --output-format csv -- python3 $R/bench.py --fmt $fmt --steps 2 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/sq_${fmt}_$i.err || exit 1
done
done
for f in fastq fasta; do for i in 1 2 3 4; do [ -d $O/sq_${f}_$i ] && KN=$([ $f = fastq ] && echo k_fq_tiles || echo k_fa_tiles) python tools/sq_table.py sq_${f}_$i; done; done > $O/sq_summary.txt
cat $O/sq_summary.txt
exit 0

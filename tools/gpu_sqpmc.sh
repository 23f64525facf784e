#!/bin/bash
# SQ counter passes over the 10 GiB FASTQ bench (one block each, separate runs).
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 5 60 rocprofv3 -L > $O/counters_list.log 2>&1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS"; do
  i=$((i+1)); rm -rf $O/sqpmc$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/sqpmc$i -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sec 0 --no-check > $O/sqpmc$i.json 2> $O/sqpmc$i.err || exit 1
done
exit 0

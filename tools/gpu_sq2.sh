#!/bin/bash
# SQ counters of the FASTQ (and FASTA) tile kernels, kernel traces of the chunkrecord builds,
# the pinned end-to-end line.  Outputs under gpurun_out/.
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
for f in fastq fasta; do
  rm -rf $O/chunk_kt_$f
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/chunk_kt_$f -o run -- python3 bench.py --kind chunkrecord --fmt $f --steps 5 --warmup 1 --no-check > $O/chunk_kt_$f.json 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --e2e --pinned --steps 3 --warmup 1 > $O/e2e_pinned.json 2>$O/e2e_pinned.err || exit 1
cat $O/e2e_pinned.json
exit 0

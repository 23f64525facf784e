#!/bin/bash
# Exploration pass: A/B of DMA cache-policy variants (FASTQ, FASTA), SQ counters of the two
# tile kernels, k_fq_tiles phase timing (diag variant), the pinned end-to-end line, the C4
# subset line with k_gather PMC.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
VARS=${VARS:-"base nt1 nt3"} ROUNDS=${ROUNDS:-2} FMT=fastq bash tools/gpu_ab.sh || exit 1
VARS=${VARS:-"base nt1 nt3"} ROUNDS=${ROUNDS:-2} FMT=fasta bash tools/gpu_ab.sh || exit 1
if [ -z "$SKIP_SQ" ]; then
i=0
for fmt in fastq fasta; do
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES"; do
  i=$((i+1)); rm -rf $O/sq_${fmt}_$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/sq_${fmt}_$i -o pmc --output-format csv -- python3 $R/bench.py --fmt $fmt --steps 2 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/sq_${fmt}_$i.err || exit 1
done
done
fi
if [ -z "$SKIP_PHASE" ]; then
SHOCKIDX_VARIANT=diag timeout -k 10 240 python -u tools/phase_timing.py > $O/phase_fastq.txt 2>&1 || exit 1
fi
if [ -n "$E2E" ]; then
timeout -k 10 300 python -u bench.py --e2e --pinned --steps 3 --warmup 1 > $O/e2e_pinned.json 2>$O/e2e_pinned.err || exit 1
fi
exit 0

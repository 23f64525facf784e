#!/bin/bash
# GPU tests of the paths given in $TESTS (default: the subset / filter / chunkrecord suites), SQ
# counters of the two tile kernels, k_fq_tiles phase timing.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
T=${TESTS:-"tests/test_gpu_subset.py tests/test_gpu_filter.py tests/test_gpu_chunk.py tests/test_gpu_part.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_sub.log 2>&1 || { tail -30 $O/pytest_sub.log; exit 1; }
tail -2 $O/pytest_sub.log
i=0
for fmt in fastq fasta; do
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES"; do
  i=$((i+1)); rm -rf $O/sq_${fmt}_$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/sq_${fmt}_$i -o pmc --output-format csv -- python3 $R/bench.py --fmt $fmt --steps 2 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/sq_${fmt}_$i.err || exit 1
done
done
SHOCKIDX_VARIANT=diag timeout -k 10 240 python -u tools/phase_timing.py > $O/phase_fastq.txt 2>&1 || exit 1
cat $O/phase_fastq.txt
exit 0

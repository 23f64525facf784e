#!/bin/bash
# SQ instruction counts of k_pipe per ablation (diag variant).  Outputs under gpurun_out/sqabl_<dbg>/.
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
for dbg in ${DBGS:-0 128 960}; do
  rm -rf $O/sqabl_$dbg
  SHOCKIDX_VARIANT=diag SHOCKIDX_DEBUG=$dbg timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM -d $O/sqabl_$dbg -o pmc --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sec 0 --no-check > $O/sqabl_$dbg.json 2> $O/sqabl_$dbg.err || exit 1
done
exit 0

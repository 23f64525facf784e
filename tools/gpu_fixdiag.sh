#!/bin/bash
# k_pipe phase breakdown + k_fixup cost by grid size (diagnostic).  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 200 python -u tools/phase_timing.py fastq 10 > $O/phase.log 2>&1 || exit 1
for g in 256 1; do
  rm -rf $O/prof_fix$g
  SHOCKIDX_FIXUP_GRID=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fix$g -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-sec 0 > $O/bench_fix$g.json 2> $O/bench_fix$g.err || exit 1
done
exit 0

#!/bin/bash
# round 5: probe of the multi-slab verify failure; 8 KiB tile variants; drop-in create with trim
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 120 python -u tools/probes/multi_verify.py > $O/multi_verify.txt 2>&1 || exit $?
for i in 1 2; do
  for v in ring0 base t8k t8kdb; do
    if [ $v = base ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
    timeout -k 10 120 python bench.py --cpu-sec 0 --warmup 30 --steps 20 --no-floor > $O/ab_${v}_$i.json 2>&1 || exit $?
  done
done
unset SHOCKIDX_VARIANT
timeout -k 10 300 python bench.py --e2e --fd --steps 6 --warmup 1 > $O/e2e_fd_keep.json 2> $O/e2e_fd_keep.err || exit $?
timeout -k 10 300 python bench.py --e2e --fd --steps 6 --warmup 1 --trim 1 > $O/e2e_fd_trim1.json 2> $O/e2e_fd_trim1.err || exit $?

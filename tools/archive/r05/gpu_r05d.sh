#!/bin/bash
# round 5: interleaved A/B of the FASTQ tile pass's VALU diet (lean), row-start layout (ring /
# ring0), opaque lane conditions (opq) and 8 workgroups per CU (…8)
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 120 python -u tools/probes/multi_verify.py > $O/multi_verify.txt 2>&1 || exit $?
for i in 1 2; do
  for v in ring0 lean0 base r0lean r0opq r0opq8 r0lean8 t8k t8kdb; do
    if [ $v = base ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
    timeout -k 10 120 python bench.py --cpu-sec 0 --warmup 30 --steps 20 --no-floor > $O/ab_${v}_$i.json 2>&1 || exit $?
  done
done

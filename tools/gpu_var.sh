#!/bin/bash
# bench the FASTQ kernels across library variants: VARS="pl6 pl8" KERNELS="stream pipe"
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
for v in ${VARS:-default}; do
  for k in ${KERNELS:-stream pipe}; do
    if [ $v = default ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
    SHOCKIDX_KERNEL=$k timeout -k 10 200 python bench.py --fmt ${FMT:-fastq} --steps ${STEPS:-20} --cpu-sec 0 > $O/var_${v}_$k.json 2>&1 || { tail -20 $O/var_${v}_$k.json; exit 1; }
    python -c "import json; d=json.load(open('$O/var_${v}_$k.json')); print('$v $k kernel_ms', d['index_kernel_ms'], 'frac', d['roofline']['frac'], 'fallbacks', d.get('lookback_selfhelp'), d['parity']['mismatches'], d['parity']['count_ok'])"
  done
done

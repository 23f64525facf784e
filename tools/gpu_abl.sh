#!/bin/bash
# tile-pass ablation variants: kernel time only (results are not checked)
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
for v in ${VARS:-abl1 abl2}; do
  SHOCKIDX_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --cpu-sec 0 --no-check > $O/abl_$v.json 2>/dev/null; rc=$?; [ $rc -gt 1 ] && exit 1
  python -c "import json; d=json.load(open('$O/abl_$v.json')); print('$v kernel_ms', d['index_kernel_ms'], 'frac', d['roofline']['frac'])"
done

#!/bin/bash
# A/B of libshockidx variants on the subset bench (BASELINE configs[3]): interleaved runs,
# gather kernel ms per run.  VARS="base v1 v2" ROUNDS=2; outputs gpurun_out/ab_subset*.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
: > $O/ab_subset.txt
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARS:-base}; do
    if [ "$v" = base ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
    timeout -k 10 240 python -u bench.py --subset --steps 10 --warmup 2 > $O/ab_subset_$v.json 2> $O/ab_subset_$v.err || { echo "variant $v failed"; tail -5 $O/ab_subset_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_subset_$v.json'));print('$v', d['gather_kernel_ms'], d['gather_kernel_ms_two_calls'], d['node_ms'], d['parity_ok'])" >> $O/ab_subset.txt
  done
done
unset SHOCKIDX_VARIANT
cat $O/ab_subset.txt

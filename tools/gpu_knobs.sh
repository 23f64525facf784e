#!/bin/bash
# tile-pass knobs (parity checked by the bench): KNOBS="name:ENV=V,ENV=V ..."
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
for spec in $KNOBS; do
  name=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -k 10 200 python bench.py --steps 20 --cpu-sec 0 > $O/knob_$name.json 2>/dev/null; rc=$?; [ $rc -gt 1 ] && exit 1
  python -c "import json; d=json.load(open('$O/knob_$name.json')); print('$name kernel_ms', d['index_kernel_ms'], 'build_ms', d['build']['kernel_ms'], 'step_ms', d['ms_per_step'], 'frac', d['roofline']['frac'], d['parity']['mismatches'], d['parity']['count_ok'])"
done

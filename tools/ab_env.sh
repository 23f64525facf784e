#!/bin/bash
# A/B of environment knobs on the 10 GiB bench (timing only).  VARIANTS="A=1:B=2 C=3" (':' joins vars)
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O; : > $O/ab_env.log
for v in ${VARIANTS}; do
  env ${v//:/ } timeout -k 10 200 python bench.py --steps 10 --cpu-sec 0 ${CHECK:---no-check} ${BENCH_ARGS} > /tmp/ab.json 2>/tmp/ab.err
  python -c "import json; d=json.loads(open('/tmp/ab.json').readline()); print('$v', 'index_ms', d['index_kernel_ms'], 'step_ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'fixups', d['fixups'], d['parity'])" >> $O/ab_env.log 2>&1 || tail -3 /tmp/ab.err >> $O/ab_env.log
done
exit 0

#!/bin/bash
# A/B of kernel variants by environment (timing only).  Outputs under gpurun_out/ab.log.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.log
for v in ${VARIANTS:-"SHOCKIDX_ONE_TILE=0" "SHOCKIDX_ONE_TILE=1"}; do
  for dbg in ${DBGS:-0}; do
    env ${v//:/ } SHOCKIDX_DEBUG=$dbg timeout -k 10 200 python bench.py --fmt ${FMT:-fastq} --size-gib ${SIZE:-10} --steps 10 --cpu-sec 0 ${CHECK:---no-check} > /tmp/ab.json 2>/tmp/ab.err
    rc=$?
    python -c "import json; d=json.loads(open('/tmp/ab.json').readline()); print('$v', 'debug', $dbg, 'index_ms', d['index_kernel_ms'], 'step_ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'parity', d['parity'])" >> gpurun_out/ab.log 2>&1 || tail -3 /tmp/ab.err >> gpurun_out/ab.log
    [ $rc -gt 1 ] && exit $rc
  done
done
exit 0

#!/bin/bash
# Phase ablation of the index kernel (timing only; results are wrong with debug bits set).
for dbg in ${DBGS:-0 1 4 5}; do
  SHOCKIDX_DEBUG=$dbg timeout -k 10 200 python bench.py --size-gib ${1:-1} --steps 10 --cpu-sec 0 --no-check > /tmp/abl.json 2>/tmp/abl.err
  python -c "import sys,json; d=json.loads(open('/tmp/abl.json').readline()); print('debug', $dbg, 'index_ms', d['index_kernel_ms'], 'step_ms', d['ms_per_step'], 'selfhelp', d['lookback_selfhelp'], 'frac', d['roofline']['frac'])" || tail -3 /tmp/abl.err
done

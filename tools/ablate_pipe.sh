#!/bin/bash
# k_pipe phase ablations (timing only; results are wrong with debug bits set).
#   64 no fold/prefix wait, 128 no validation, 256 no newline array + no validation,
#   512 no row stores, 960 = only load + stage + count publish
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O; : > $O/ablate_pipe.log
for dbg in ${DBGS:-0 64 128 256 512 576 960}; do
  SHOCKIDX_DEBUG=$dbg timeout -k 10 200 python bench.py --steps 10 --cpu-sec 0 --no-check > /tmp/abl.json 2>/tmp/abl.err
  python -c "import json; d=json.loads(open('/tmp/abl.json').readline()); print('debug', $dbg, 'index_ms', d['index_kernel_ms'], 'step_ms', d['ms_per_step'], 'frac', d['roofline']['frac'])" >> $O/ablate_pipe.log 2>&1 || tail -3 /tmp/abl.err >> $O/ablate_pipe.log
done
exit 0

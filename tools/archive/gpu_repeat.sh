#!/bin/bash
# The default bench line five times back to back in one call (fresh box): how often the slow
# state shows (profiles/r04/slow_state/).
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/repeat; mkdir -p $O
for r in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --cpu-sec 0 > $O/bench_$r.json 2> $O/bench_$r.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_$r.json'));print($r, d['value'], d['index_kernel_ms'], d['build']['frac'], d['box_floor']['ms'])"
done
exit 0

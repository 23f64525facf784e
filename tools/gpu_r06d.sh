#!/bin/bash
# Round-6: the drop-in's end-to-end fd build with the shim's per-call trim, whole-node layout
# against the two-slot layout (a device cap), each twice, on one box.
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --e2e --fd --trim 1 --steps 3 --warmup 1 > $O/e2e_trim1_whole_$i.json 2> $O/e1_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --e2e --fd --trim 1 --dev-cap 4 --steps 3 --warmup 1 > $O/e2e_trim1_cap4_$i.json 2> $O/e2_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/e2e_whole_$i.json 2> $O/e3_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --e2e --fd --dev-cap 4 --steps 3 --warmup 1 > $O/e2e_cap4_$i.json 2> $O/e4_$i.err || exit 1
done
for f in $O/e2e_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d.get('create_gib_s'), d['timings_ms']['h2d_ms'], d.get('build_path'), d.get('workspace_bytes_after_last_call'))"; done

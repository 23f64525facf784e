#!/bin/bash
# k_stream phase ablations (SIDX_DIAG variant): bench --no-check per SHOCKIDX_DEBUG mask.
#   64 no folds | 128 no validation | 256 no newline array (+ no validation) | 512 no row stores
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
: > $O/abl_stream.txt
for dbg in 0 512 128 256 320 64; do
  SHOCKIDX_VARIANT=${VAR:-diag} SHOCKIDX_DEBUG=$dbg timeout -k 10 200 python bench.py --steps 10 --cpu-sec 0 --no-check > /tmp/abl.json 2>/tmp/abl.err; rc=$?; [ $rc -gt 1 ] && { cat /tmp/abl.err; exit 1; }
  python -c "import json; d=json.load(open('/tmp/abl.json')); print('debug', $dbg, 'kernel_ms', d['index_kernel_ms'], 'frac', d['roofline']['frac'])" >> $O/abl_stream.txt
done
timeout -k 10 200 python bench.py --steps 10 --cpu-sec 0 > /tmp/abl.json 2>/tmp/abl.err || { cat /tmp/abl.err; exit 1; }
python -c "import json; d=json.load(open('/tmp/abl.json')); print('production kernel_ms', d['index_kernel_ms'], 'frac', d['roofline']['frac'], 'parity', d['parity'])" >> $O/abl_stream.txt
cat $O/abl_stream.txt

#!/bin/bash
# Round-6 late calls: the capped build's slab-local errors (tests/test_gpu_ring.py) and the FASTA
# tile-pass variants (tools/probes/fa2slot_variant.py, fa_early_variant.py) in one process A/B.
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
e=0
if [ -z "$SKIP_RING" ]; then
  timeout -k 10 700 python -u -m pytest tests/test_gpu_ring.py -v --timeout 300 --timeout-method thread > $O/ring.log 2>&1
  e=$?
  tail -15 $O/ring.log
  case $e in 0|1) ;; *) exit $e ;; esac  # a crash, abort or time limit: nothing more on the GPU
fi
timeout -k 10 400 python -u tools/ab_inproc.py base ${AB_VARIANTS:-fa2slot faearly} --fmt ${AB_FMT:-fasta} --copies ${AB_COPIES:-2} --check-rows > $O/ab_${AB_FMT:-fasta}.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab_${AB_FMT:-fasta}.json
exit $e

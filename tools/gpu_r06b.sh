#!/bin/bash
# Round-6 late calls: the capped build's slab-local errors (tests/test_gpu_ring.py) and the FASTA
# tile-pass variants (tools/probes/fa2slot_variant.py, fa_early_variant.py) in one process A/B.
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_ring.py -v --timeout 300 --timeout-method thread > $O/ring.log 2>&1
e=$?
tail -15 $O/ring.log
case $e in 0|1) ;; *) exit $e ;; esac  # a crash, abort or time limit: nothing more on the GPU
timeout -k 10 400 python -u tools/ab_inproc.py base ${AB_VARIANTS:-fa2slot faearly} --fmt fasta --copies 2 --check-rows > $O/ab_fa.json 2> $O/ab_fa.err || { tail -5 $O/ab_fa.err; exit 1; }
cat $O/ab_fa.json
exit $e

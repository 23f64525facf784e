#!/bin/bash
# FASTQ tile pass: the last record's end in the starts' store instruction (base) vs its own store
# (endsep) -- parity, the FASTQ GPU tests, then A/B fresh and after the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --cpu-sec 0 --no-floor > $O/em_check.json 2> $O/em_check.err || { tail -5 $O/em_check.err; exit 1; }
python -c "import json;d=json.load(open('$O/em_check.json'));print(d['parity'])"
VARS="base endsep" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_endmerge_fresh.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/em_suite.log 2>&1 || { tail -20 $O/em_suite.log; exit 1; }
tail -1 $O/em_suite.log
VARS="base endsep" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_endmerge_after.txt
exit 0

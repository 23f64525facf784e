#!/bin/bash
# FASTQ row starts stored non-temporally (ntst) vs as built, fresh and after the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
SHOCKIDX_VARIANT=ntst timeout -k 10 300 python bench.py --steps 5 --warmup 3 --cpu-sec 0 --no-floor > $O/ntst_check.json 2> $O/ntst_check.err || { tail -5 $O/ntst_check.err; exit 1; }
python -c "import json;d=json.load(open('$O/ntst_check.json'));print(d['parity'])"
VARS="base ntst" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_ntst_fresh.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/ntst_suite.log 2>&1 || exit 1
VARS="base ntst" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_ntst_after.txt
exit 0

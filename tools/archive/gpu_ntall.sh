#!/bin/bash
# Tile words and line positions stored non-temporally too (ntall) vs as built (row starts nt):
# parity, then A/B of the FASTQ and line builds, fresh and after the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
for k in "--fmt fastq" "--kind line"; do
  SHOCKIDX_VARIANT=ntall timeout -k 10 300 python bench.py $k --steps 5 --warmup 3 --cpu-sec 0 --no-floor > $O/ntall_check.json 2> $O/ntall_check.err || { tail -5 $O/ntall_check.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ntall_check.json'));print('$k', d.get('parity', d.get('parity_ok')))"
done
ab() {
  VARS="base ntall" ROUNDS=2 bash tools/gpu_ab.sh || return 1
  cp $O/ab_fastq.txt $O/ab_ntall_fastq_$1.txt
  KIND=line VARS="base ntall" ROUNDS=2 bash tools/gpu_ab.sh || return 1
  cp $O/ab_fastq.txt $O/ab_ntall_line_$1.txt
}
ab fresh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/ntall_suite.log 2>&1 || { tail -20 $O/ntall_suite.log; exit 1; }
tail -1 $O/ntall_suite.log
ab after || exit 1
cat $O/ab_ntall_*_fresh.txt $O/ab_ntall_*_after.txt
exit 0

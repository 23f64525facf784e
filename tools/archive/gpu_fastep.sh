#!/bin/bash
# k_fa_anon_write step size: the FASTA / SAM anonymize GPU tests on the default build, then an
# interleaved A/B of 4 KiB steps (base) vs 1 KiB (fa1) and 2 KiB (fa2), and per-kernel times.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/fastep; mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_filter.py -k "anonymize" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
[ -n "$NOTEST" ] || tail -3 $O/pytest.log
VARS="${VARS:-base fa1 fa2}" ROUNDS=3 KIND=filter FILTER=anonymize FMT=fasta timeout -k 10 600 bash tools/gpu_ab.sh || exit 1
for v in ${KT:-base fa1}; do
  rm -rf $O/kt_$v
  if [ $v = base ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- python3 $R/bench.py --kind filter --fmt fasta --filter anonymize --steps 5 --warmup 1 --cpu-sec 0 > $O/$v.json 2> $O/$v.err || exit 1
  python - "$O/kt_$v" "$v" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0])))
print(sys.argv[2], [(r["Name"][:28], round(float(r["AverageNs"]) / 1e3, 1)) for r in rows if "k_fa" in r["Name"]])
PY
done
exit 0

#!/bin/bash
# FASTA anonymize writer: as built vs without its global stores (ablF1), per-kernel times.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/faabl; mkdir -p $O
for v in base ablF1; do
  rm -rf $O/kt_$v
  if [ $v = base ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- python3 $R/bench.py --kind filter --fmt fasta --filter anonymize --steps 5 --warmup 1 --cpu-sec 0 > $O/$v.json 2> $O/$v.err
  python - "$O/kt_$v" "$v" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0])))
print(sys.argv[2], [(r["Name"][:28], round(float(r["AverageNs"]) / 1e3, 1)) for r in rows if "anon" in r["Name"]])
PY
done
unset SHOCKIDX_VARIANT
exit 0

#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of k_fq_tiles for the default library and VARS variants (one PMC pass each)
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
for v in default ${VARS}; do
  if [ $v = default ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pf_${v}_$c
    timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pf_${v}_$c -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2>&1 || exit 1
  done
  V=$v python3 - <<'PY'
import csv, glob, os
v = os.environ["V"]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = {}
    for p in glob.glob(f"gpurun_out/pf_{v}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "k_fq_tiles" in r["Kernel_Name"] and r["Counter_Name"] == c:
                k = r.get("Dispatch_Id")
                per[k] = per.get(k, 0) + float(r["Counter_Value"])
    vals = list(per.values())
    kib = sum(vals) / len(vals)
    b = (2 if c == "FETCH_SIZE" else 1) * kib * 1024
    print(v, c, f"{b / 1e9:.3f} GB per launch", f"({b / (10 << 30):.4f} x input)" if c == "FETCH_SIZE" else "")
PY
done

#!/bin/bash
# The effective shader clock of k_fq_tiles fresh and after two minutes of GPU load (the suite).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
clk() {
  O=$R/gpurun_out/clock_$1; rm -rf $O; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --cpu-sec 0 > $O/bench.json 2> $O/bench.err || return 1
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/grbm -o pmc --output-format csv -- python3 $R/bench.py --steps 10 --warmup 100 --cpu-sec 0 --no-check > /dev/null 2> $O/grbm.err || return 1
  python - "$O" <<'PY'
import csv, glob, json, sys
O = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(O + "/grbm/**/*counter_collection.csv", recursive=True)[0])))
by = {}
for r in rows:
    if "k_fq_tiles" in r["Kernel_Name"]:
        by.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
act = sum(v.get("GRBM_GUI_ACTIVE", 0) for v in by.values()) / len(by)
kt = list(csv.DictReader(open(glob.glob(O + "/kt/**/*kernel_stats.csv", recursive=True)[0])))
ns = [float(r["AverageNs"]) for r in kt if "k_fq_tiles" in r["Name"]][0]
fl = [float(r["AverageNs"]) for r in kt if "k_stream_floor" in r["Name"]][0]
out = {"k_fq_tiles_ns": ns, "k_stream_floor_ns": fl, "grbm_gui_active_per_dispatch": act, "mhz_per_xcd": act / ns * 1e3 / 8}
print(O.split("/")[-1], json.dumps(out))
json.dump(out, open(O + "/clock.json", "w"))
PY
}
clk fresh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/clock_suite.log 2>&1 || exit 1
clk after_suite || exit 1
exit 0

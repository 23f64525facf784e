#!/bin/bash
# Effective shader clock of the FASTQ build on this box: GRBM_GUI_ACTIVE (GPU busy cycles) per
# k_fq_tiles dispatch over its duration, next to the box's streaming floor in the bench line.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/clock; mkdir -p $O
rm -rf $O/kt $O/grbm
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --cpu-sec 0 > $O/bench.json 2> $O/bench.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/grbm -o pmc --output-format csv -- python3 $R/bench.py --steps 10 --warmup 100 --cpu-sec 0 --no-check > /dev/null 2> $O/grbm.err || exit 1
python - "$O" <<'PY'
import csv, glob, json, sys
O = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(O + "/grbm/**/*counter_collection.csv", recursive=True)[0])))
by = {}
for r in rows:
    if "k_fq_tiles" not in r["Kernel_Name"]:
        continue
    by.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
act = [v.get("GRBM_GUI_ACTIVE", 0) for v in by.values()]
cnt = [v.get("GRBM_COUNT", 0) for v in by.values()]
kt = list(csv.DictReader(open(glob.glob(O + "/kt/**/*kernel_stats.csv", recursive=True)[0])))
avg_ns = [float(r["AverageNs"]) for r in kt if "k_fq_tiles" in r["Name"]][0]
b = json.load(open(O + "/bench.json"))
out = {"dispatches": len(act), "grbm_gui_active_avg": sum(act) / len(act), "grbm_count_avg": sum(cnt) / len(cnt),
       "k_fq_tiles_avg_ns_kernel_trace": avg_ns,
       "clock_mhz_gui_active_over_trace": sum(act) / len(act) / avg_ns * 1e3,
       "bench_index_kernel_ms": b["index_kernel_ms"], "box_floor": b.get("box_floor")}
print(json.dumps(out))
json.dump(out, open(O + "/clock.json", "w"))
PY

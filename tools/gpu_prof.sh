#!/bin/bash
# rocprofv3 kernel stats of the default bench (SHOCKIDX_KERNEL from the caller's env)
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
rm -rf $O/prof_${TAG:-x}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG:-x} -o run -- python3 bench.py --steps 20 --cpu-sec 0 > $O/prof_${TAG:-x}.json 2>&1 || { tail -20 $O/prof_${TAG:-x}.json; exit 1; }
f=$(find $O/prof_${TAG:-x} -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f} total_ms {float(r["TotalDurationNs"])/1e6:8.2f}')
PY

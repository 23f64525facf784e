#!/bin/bash
# phase stamps (SIDX_DIAG variant) + SQ counters for k_pipe and k_stream
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
for k in pipe stream; do
  SHOCKIDX_KERNEL=$k SHOCKIDX_VARIANT=diag timeout -k 10 200 python -u tools/phase_timing.py fastq 10 > $O/ph_$k.txt 2>&1 || { tail $O/ph_$k.txt; exit 1; }
  cat $O/ph_$k.txt
done
for k in pipe stream; do
rm -rf $O/sq_$k; SHOCKIDX_KERNEL=$k timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY -d $O/sq_$k -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2>&1 || exit 1
K=$k python3 - <<'PY'
import csv, glob, collections, os
k = os.environ["K"]
agg = collections.defaultdict(list)
for p in glob.glob(f"gpurun_out/sq_{k}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if f"k_{k}" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(k)
for c, v in sorted(agg.items()):
    print(f"   {c:24s} {sum(v)/len(v):.4e}")
PY
done

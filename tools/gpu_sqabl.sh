#!/bin/bash
# instruction counts per ablation (SIDX_DIAG variant), k_pipe and k_stream
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
: > $O/sqabl.txt
for k in pipe stream; do
for dbg in 0 128 256 512 896; do
rm -rf $O/sqa; SHOCKIDX_VARIANT=diag SHOCKIDX_DEBUG=$dbg SHOCKIDX_KERNEL=$k timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY -d $O/sqa -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2>&1; rc=$?; [ $rc -gt 1 ] && exit 1
K=$k D=$dbg python3 - >> $O/sqabl.txt <<'PY'
import csv, glob, collections, os
k = os.environ["K"]
agg = collections.defaultdict(list)
for p in glob.glob("gpurun_out/sqa/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if f"k_{k}" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(k, "debug", os.environ["D"], " ".join(f"{c.replace('SQ_','')}={sum(v)/len(v):.3e}" for c, v in sorted(agg.items())))
PY
done
done
cat $O/sqabl.txt

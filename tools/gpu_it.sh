#!/bin/bash
# iteration loop for the FASTQ kernels: parity (stream + pipe), bench, SQ counters
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_scale.py"}
for k in ${KERNELS:-stream pipe}; do
  SHOCKIDX_KERNEL=$k timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread -k "${TESTK:-not two_contexts}" > $O/it_pytest_$k.log 2>&1 || { tail -30 $O/it_pytest_$k.log; exit 1; }
  echo "$k: $(tail -1 $O/it_pytest_$k.log)"
done
for k in ${KERNELS:-stream pipe}; do
  SHOCKIDX_KERNEL=$k timeout -k 10 200 python bench.py --steps 20 --cpu-sec 0 > $O/it_bench_$k.json 2>&1 || { tail $O/it_bench_$k.json; exit 1; }
  python -c "import json; d=json.load(open('$O/it_bench_$k.json')); print('$k kernel_ms', d['index_kernel_ms'], 'frac', d['roofline']['frac'], 'fallbacks', d.get('lookback_selfhelp'), d['parity'])"
done
for k in ${KERNELS:-stream pipe}; do
rm -rf $O/sqi; SHOCKIDX_KERNEL=$k timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY -d $O/sqi -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2>&1; rc=$?; [ $rc -gt 1 ] && exit 1
K=$k python3 - <<'PY'
import csv, glob, collections, os
k = os.environ["K"]
agg = collections.defaultdict(list)
for p in glob.glob("gpurun_out/sqi/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if f"k_{k}" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(k, " ".join(f"{c.replace('SQ_','')}={sum(v)/len(v):.3e}" for c, v in sorted(agg.items())))
PY
done

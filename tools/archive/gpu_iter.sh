#!/bin/bash
# Iteration pass on the GPU box: the -m gpu suite (or TESTS=<pytest args>), then the default
# FASTQ bench line and a kernel trace of it.  Outputs: gpurun_out/it_*.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 300 --timeout-method thread > $O/it_pytest.log 2>&1 || { tail -30 $O/it_pytest.log; exit 1; }
  tail -2 $O/it_pytest.log
fi
for f in ${FMTS:-fastq}; do
  rm -rf $O/it_kt_$f
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/it_kt_$f -o kt --output-format csv -- python3 bench.py --fmt $f --steps 20 --warmup 3 --cpu-sec 0 ${BENCH_ARGS} > $O/it_bench_$f.json 2> $O/it_bench_$f.err || { tail -5 $O/it_bench_$f.err; exit 1; }
  python3 - $O/it_kt_$f/kt_kernel_stats.csv <<'PY'
import csv,sys
for x in csv.DictReader(open(sys.argv[1])):
    if float(x['Percentage'])>0.01: print(x['Name'][:48], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us')
PY
  head -c 900 $O/it_bench_$f.json; echo
done
exit 0

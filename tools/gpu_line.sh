#!/bin/bash
# line index: tile-pass GPU parity, bench lines (tile pass and two-pass), kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
TAG=${TAG:-line}
timeout -k 10 600 python -u -m pytest tests/test_gpu_line.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > $O/${TAG}_pytest.log 2>&1 || { tail -30 $O/${TAG}_pytest.log; exit 1; }
echo "pytest: $(tail -1 $O/${TAG}_pytest.log)"
for f in fastq fasta; do
  timeout -k 10 300 python -u bench.py --kind line --fmt $f --steps ${STEPS:-10} --warmup 2 > $O/${TAG}_bench_$f.json 2> $O/${TAG}_bench_$f.err || { tail $O/${TAG}_bench_$f.err; exit 1; }
  cat $O/${TAG}_bench_$f.json
done
SHOCKIDX_LINE_MODE=two timeout -k 10 300 python -u bench.py --kind line --fmt fastq --steps ${STEPS:-10} --warmup 2 > $O/${TAG}_bench_two.json 2> $O/${TAG}_bench_two.err || { tail $O/${TAG}_bench_two.err; exit 1; }
cat $O/${TAG}_bench_two.json
if [ -n "$PROF" ]; then
  rm -rf $O/${TAG}_kt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_kt -o run -- python3 bench.py --kind line --fmt fastq --steps 5 --warmup 1 > /dev/null 2>&1 || exit 1
  cp "$(find $O/${TAG}_kt -name '*kernel_stats.csv' -print -quit)" $O/${TAG}_kernel_stats.csv
fi

#!/bin/bash
# chunkrecord: GPU parity (speculative + serial), 10 GiB bench lines with whole-table oracle
# parity, kernel stats.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
TAG=${TAG:-chunk}
timeout -k 10 600 python -u -m pytest tests/test_gpu_chunk.py -x -q --timeout 300 --timeout-method thread \
  > $O/${TAG}_pytest.log 2>&1 || { tail -30 $O/${TAG}_pytest.log; exit 1; }
echo "pytest: $(tail -1 $O/${TAG}_pytest.log)"
for f in fastq fasta; do
  timeout -k 10 300 python -u bench.py --kind chunkrecord --fmt $f --steps ${STEPS:-5} --warmup 2 > $O/${TAG}_bench_$f.json 2> $O/${TAG}_bench_$f.err || { tail $O/${TAG}_bench_$f.err; exit 1; }
  cat $O/${TAG}_bench_$f.json
done
if [ -n "$PROF" ]; then
  for f in fastq fasta; do
    rm -rf $O/${TAG}_kt_$f
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_kt_$f -o run -- python3 bench.py --kind chunkrecord --fmt $f --steps 5 --warmup 1 --no-check > /dev/null 2>&1 || exit 1
  done
fi
exit 0

#!/bin/bash
# Closing check after the filter writer changes (sidx_filter.hip only; the tile kernels and their
# PMC summaries are unchanged): the whole GPU suite, smoke, the FASTQ filter lines and the default bench.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/close2; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
for f in fq2fa anonymize; do
  timeout -k 10 300 python -u bench.py --kind filter --fmt fastq --filter $f --steps 20 --warmup 3 > $O/bench_filter_fastq_$f.json 2> $O/bench_filter_fastq_$f.err || exit 1
done
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cat $O/bench_default.json
exit 0

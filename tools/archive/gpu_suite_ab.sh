#!/bin/bash
# The whole -m gpu suite, then interleaved A/Bs of libshockidx variants ($VARS) for each format in
# $FMTS, then the line bench.  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
for f in ${FMTS:-fastq fasta}; do
  VARS=${VARS:-base} ROUNDS=${ROUNDS:-3} FMT=$f bash tools/gpu_ab.sh || exit 1
done
timeout -k 10 300 python -u bench.py --kind line --cpu-sec 0 > $O/bench_line.json 2> $O/bench_line.err || exit 1
python -c "import json;d=json.load(open('$O/bench_line.json'));print('line', d['index_kernel_ms'], d['build']['kernel_ms'], d['ms_per_step'], d['parity_ok'])"
exit 0

#!/bin/bash
# Round 4, late: the narrow line-position layout -- the GPU tests of every path built on the line
# pass, then the line build A/B against the previous layout (lold) and the line bench line; FASTA
# anonymize with its boundaries from the record index vs the scan.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_line.py tests/test_gpu_sam.py tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_subset.py tests/test_gpu_fdpipe.py tests/test_gpu_filter.py -x -q --timeout 300 --timeout-method thread > $O/r04d_tests.log 2>&1 || { tail -30 $O/r04d_tests.log; exit 1; }
tail -2 $O/r04d_tests.log
KIND=line VARS="base lold" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 python bench.py --kind line --cpu-sec 0 > $O/line_narrow.json 2> $O/line_narrow.err || exit 1
cat $O/line_narrow.json
timeout -k 10 300 python bench.py --kind filter --fmt fasta --filter anonymize --steps 5 --warmup 1 > $O/fa_anon_index.json 2> $O/fa_anon_index.err || exit 1
SHOCKIDX_ANON_SCAN=1 timeout -k 10 300 python bench.py --kind filter --fmt fasta --filter anonymize --steps 5 --warmup 1 --cpu-sec 0 > $O/fa_anon_scan.json 2> $O/fa_anon_scan.err || exit 1
cat $O/fa_anon_index.json $O/fa_anon_scan.json
exit 0

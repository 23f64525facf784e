#!/bin/bash
# Round 4, late: the FASTQ tile body and halo pieces in one DMA statement (base) vs the body alone
# under one M0 (nofold) vs one M0 per piece (m0off) -- parity with the bench row checks, the tile
# pass tests, then A/B.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --cpu-sec 0 --no-floor > $O/fold_check.json 2> $O/fold_check.err || { tail -5 $O/fold_check.err; exit 1; }
python -c "import json;d=json.load(open('$O/fold_check.json'));print(d['parity'], d['index_kernel_ms'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_slabs.py -x -q --timeout 300 --timeout-method thread > $O/r04h_tests.log 2>&1 || { tail -30 $O/r04h_tests.log; exit 1; }
tail -1 $O/r04h_tests.log
VARS="base nofold m0off" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_halofold_fastq.txt
exit 0

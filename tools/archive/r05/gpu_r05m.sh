#!/bin/bash
# round 5: the deferred tile-pass stores -- A/B over 6 input copies, then the FASTQ parity suites
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 500 python -u tools/ab_inproc.py base nodefer ring0 dfl0 abl4 --copies 6 --rounds 3 --per 5 --warmup 5 > $O/ab_fq.json 2> $O/ab_fq.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_integrity.py tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_fdpipe.py tests/test_gpu_filter.py tests/test_gpu_multi.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log

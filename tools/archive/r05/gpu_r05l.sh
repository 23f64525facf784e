#!/bin/bash
# round 5: (1) FASTQ: the tile pass's stores issued after the next tile's DMA (defer), against
# the same without (nodefer), the round-4 kernel (ring0) and no row-start stores at all (abl4),
# over 6 input copies; (2) FASTA ablations; (3) the FASTQ-side parity suites on the new default
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 500 python -u tools/ab_inproc.py base nodefer ring0 dfl0 abl4 --copies 6 --rounds 3 --per 5 --warmup 5 > $O/ab_fq.json 2> $O/ab_fq.err || exit $?
timeout -k 10 500 python -u tools/ab_inproc.py base faA1 faA2 faA3 --fmt fasta --copies 4 --rounds 4 --per 8 --warmup 8 > $O/ab_fa.json 2> $O/ab_fa.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_integrity.py tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_fdpipe.py tests/test_gpu_filter.py tests/test_gpu_multi.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log

#!/bin/bash
# round 5: (1) FASTQ store wave (sw: one wave issues every global store and never waits on a
# DMA) over 6 input copies; (2) FASTA / line stores deferred past the next DMA (default) against
# not; (3) parity suites on the default build
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 500 python -u tools/ab_inproc.py ring0 base sw swl0 abl4 --copies 6 --rounds 3 --per 5 --warmup 5 > $O/ab_fq.json 2> $O/ab_fq.err || exit $?
timeout -k 10 400 python -u tools/ab_inproc.py base fnodefer --fmt fasta --copies 4 --rounds 4 --per 8 --warmup 8 > $O/ab_fa.json 2> $O/ab_fa.err || exit $?
timeout -k 10 400 python -u tools/ab_inproc.py base lnodefer --kind line --copies 4 --rounds 4 --per 8 --warmup 8 > $O/ab_line.json 2> $O/ab_line.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_integrity.py tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_fdpipe.py tests/test_gpu_fasta_tiles.py tests/test_gpu_line.py tests/test_gpu_multi.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log

#!/bin/bash
# The drop-in path as committed (page-cache DMA, all chunks pinned for the build): the fd / host
# GPU tests in both producer modes, then the end-to-end bench lines.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fdpipe.py tests/test_gpu_host.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $O/mmap3_tests.log 2>&1 || { tail -30 $O/mmap3_tests.log; exit 1; }
tail -1 $O/mmap3_tests.log
SHOCKIDX_NO_MMAP_DMA=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fdpipe.py -x -q --timeout 300 --timeout-method thread > $O/mmap3_tests2.log 2>&1 || { tail -30 $O/mmap3_tests2.log; exit 1; }
tail -1 $O/mmap3_tests2.log
timeout -k 10 400 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/bench_e2e_fastq_fd.json 2> $O/bench_e2e_fd.err || exit 1
timeout -k 10 400 python -u bench.py --e2e --fd --fmt fasta --steps 3 --warmup 1 > $O/bench_e2e_fasta_fd.json 2> $O/bench_e2e_fasta_fd.err || exit 1
timeout -k 10 400 python -u bench.py --e2e --pinned --steps 3 --warmup 1 > $O/bench_e2e_fastq_pinned.json 2> $O/bench_e2e_pinned.err || exit 1
for f in bench_e2e_fastq_fd bench_e2e_fasta_fd bench_e2e_fastq_pinned; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d.get('create_gib_s'), d['timings_ms'])"; done
exit 0

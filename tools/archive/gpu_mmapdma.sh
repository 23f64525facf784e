#!/bin/bash
# The drop-in path's producer: DMA straight out of the page cache (default) vs pread into pinned
# staging (SHOCKIDX_NO_MMAP_DMA) -- the fd pipeline tests in both modes, then the e2e bench, twice each.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fdpipe.py tests/test_gpu_host.py -x -q --timeout 300 --timeout-method thread > $O/mmap_tests.log 2>&1 || { tail -30 $O/mmap_tests.log; exit 1; }
tail -1 $O/mmap_tests.log
SHOCKIDX_NO_MMAP_DMA=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fdpipe.py -x -q --timeout 300 --timeout-method thread > $O/mmap_tests2.log 2>&1 || { tail -30 $O/mmap_tests2.log; exit 1; }
tail -1 $O/mmap_tests2.log
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/e2e_fd_mmap_$r.json 2> $O/e2e_fd_mmap_$r.err || exit 1
  SHOCKIDX_NO_MMAP_DMA=1 timeout -k 10 400 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/e2e_fd_pread_$r.json 2> $O/e2e_fd_pread_$r.err || exit 1
  for m in mmap pread; do python -c "import json;d=json.load(open('$O/e2e_fd_${m}_$r.json'));print('$m', d['value'], d['create_gib_s'], d['timings_ms'])"; done
done
exit 0

#!/bin/bash
# Page-cache staging on every fd path (one-pass build_fd / create, chunkrecord_fd, multi-GPU slab
# staging): their GPU tests with it and with the pread staging (SHOCKIDX_NO_MMAP_DMA).
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
T="tests/test_gpu_fdpipe.py tests/test_gpu_host.py tests/test_gpu_multi.py tests/test_gpu_chunk.py tests/test_gpu_scale.py"
timeout -k 10 900 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > $O/stagefd_tests.log 2>&1 || { tail -30 $O/stagefd_tests.log; exit 1; }
tail -1 $O/stagefd_tests.log
SHOCKIDX_NO_MMAP_DMA=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_fdpipe.py tests/test_gpu_multi.py tests/test_gpu_chunk.py -x -q --timeout 300 --timeout-method thread > $O/stagefd_tests2.log 2>&1 || { tail -30 $O/stagefd_tests2.log; exit 1; }
tail -1 $O/stagefd_tests2.log
exit 0

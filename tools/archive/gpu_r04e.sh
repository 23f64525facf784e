#!/bin/bash
# Round 4, late: packed per-workgroup position arrays in the line pass -- the GPU tests of the
# paths on it, then the A/B against the fixed per-tile slots (lslot) and the no-store ablation.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_line.py tests/test_gpu_sam.py tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_subset.py tests/test_gpu_fdpipe.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $O/r04e_tests.log 2>&1 || { tail -30 $O/r04e_tests.log; exit 1; }
tail -2 $O/r04e_tests.log
KIND=line VARS="base lslot ablL1" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
exit 0

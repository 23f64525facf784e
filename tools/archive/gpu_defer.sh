#!/bin/bash
# Tile stores held over the next tile's DMA: the record / filter GPU tests, then interleaved A/Bs
# of the default build (held) against a variant that stores in place ($VAR), per format.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/defer; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_filter.py} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for f in ${FMTS:-fastq}; do
  VARS="base ${VAR:-fqd0}" ROUNDS=${ROUNDS:-4} KIND=${KIND:-record} FMT=$f timeout -k 10 600 bash tools/gpu_ab.sh > $O/ab_$f.txt || { cat $O/ab_$f.txt; exit 1; }
  cat $O/ab_$f.txt
done
exit 0

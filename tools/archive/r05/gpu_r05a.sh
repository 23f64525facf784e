#!/bin/bash
# round 5, first GPU pass: integrity + parity suites on the ring-store kernel, default bench,
# then an interleaved A/B of the FASTQ row-start stores (ring vs the round-4 fixed slots)
set -o pipefail
mkdir -p gpurun_out/r05a
O=gpurun_out/r05a
timeout -k 10 900 python -u -m pytest tests/test_gpu_integrity.py tests/test_gpu_multi.py tests/test_gpu_parity.py \
  tests/test_gpu_fdpipe.py tests/test_gpu_slabs.py tests/test_gpu_filter.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
for i in 1 2; do
  SHOCKIDX_VARIANT=ring0 timeout -k 10 120 python bench.py --cpu-sec 0 --warmup 30 --steps 20 > $O/ab_ring0_$i.json 2>&1 || exit $?
  timeout -k 10 120 python bench.py --cpu-sec 0 --warmup 30 --steps 20 > $O/ab_ring_$i.json 2>&1 || exit $?
  SHOCKIDX_VARIANT=db1 timeout -k 10 120 python bench.py --cpu-sec 0 --warmup 30 --steps 20 > $O/ab_db1_$i.json 2>&1 || exit $?
done

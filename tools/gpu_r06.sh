#!/bin/bash
# Round-6 GPU calls (run on the box by gpurun; outputs under gpurun_out/$CALL/).
#  CALL=a: the dense-line FASTQ variants (SIDX_FQ_DENSE): parity suite on the variant, the in-process A/B
#          over 4 input copies with whole-table hashes, and the hunt for the ID-compare experiment's input
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); CALL=${CALL:-a}; O=$R/gpurun_out/$CALL; mkdir -p $O
step() { echo "== $* ($(date +%T))"; }
if [ "$CALL" = b ]; then
  step list-avail
  timeout -s KILL 120 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || { tail -5 $O/list_avail.txt; exit 1; }
  grep -c "" $O/list_avail.txt
  step suite
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  grep -E "GiB/s end to end" $O/pytest_gpu.log
  step driver-bench
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { tail -20 $O/bench_driver_cmd.err; exit 1; }
  cat $O/bench_driver_cmd.json
  step copies
  timeout -k 10 300 python -u tools/probes/copy_pmc.py --copies 4 --per 4 > $O/copies.json 2> $O/copies.err || { tail -20 $O/copies.err; exit 1; }
  cat $O/copies.json
  exit 0
fi
if [ "$CALL" = a ]; then
  step parity-dense
  SHOCKIDX_VARIANT=dense timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_dense.log 2>&1 || { tail -30 $O/pytest_dense.log; exit 1; }
  tail -1 $O/pytest_dense.log
  step ab
  timeout -k 10 600 python -u tools/ab_inproc.py base dense densent --copies 4 --rounds 4 --per 5 --turn-warmup 20 --check-rows > $O/ab_fq.json 2> $O/ab_fq.err || { tail -20 $O/ab_fq.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ab_fq.json'));print({k:(v['k_med'],v['b_med'],v['count_ok']) for k,v in d['ab'].items()}, d['rows_agree'])"
  step idc-hunt
  SHOCKIDX_VARIANT=idc timeout -k 10 400 python -u tools/probes/idc_hunt.py --seeds 1 2 --cuts 48 --out $O/idc > $O/idc_hunt.jsonl 2> $O/idc_hunt.err || { tail -20 $O/idc_hunt.err; exit 1; }
  tail -3 $O/idc_hunt.jsonl
  step ring-tests
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_fdpipe.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_ring.log 2>&1 || { tail -40 $O/pytest_ring.log; exit 1; }
  tail -3 $O/pytest_ring.log
  step cap-10gib
  timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v -s -k "2gib_cap" --timeout 500 --timeout-method thread > $O/pytest_cap.log 2>&1 || { tail -40 $O/pytest_cap.log; exit 1; }
  grep -E "GiB/s|passed|failed" $O/pytest_cap.log
  exit 0
fi

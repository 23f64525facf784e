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
if [ "$CALL" = c ]; then  # the rest of the suite after b's stop, the driver's bench, per-copy timing and counters
  step suite-rest
  timeout -k 10 800 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_sam.py tests/test_gpu_scale.py tests/test_gpu_slabs.py tests/test_gpu_subset.py -m gpu -x -v -s --timeout 600 --timeout-method thread > $O/pytest_rest.log 2>&1 || { tail -40 $O/pytest_rest.log; exit 1; }
  tail -2 $O/pytest_rest.log
  grep -E "GiB/s end to end" $O/pytest_rest.log
  step driver-bench
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { tail -20 $O/bench_driver_cmd.err; exit 1; }
  cat $O/bench_driver_cmd.json
  step copies
  timeout -k 10 300 python -u tools/probes/copy_pmc.py --copies 4 --per 4 > $O/copies.json 2> $O/copies.err || { tail -20 $O/copies.err; exit 1; }
  cat $O/copies.json
  i=0
  for set in "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum" \
             "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE" \
             "TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum" \
             "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum"; do
    i=$((i+1)); rm -rf $O/pmc_$i
    step pmc-$i
    timeout -s KILL 240 rocprofv3 --pmc $set -d $O/pmc_$i -o pmc --output-format csv -- python3 $R/tools/probes/copy_pmc.py --copies 4 --per 3 > $O/pmc_run_$i.json 2> $O/pmc_run_$i.err || { tail -5 $O/pmc_run_$i.err; exit 1; }
    python tools/probes/copy_pmc.py --summarize $O/pmc_$i $O/pmc_run_$i.json > $O/pmc_sum_$i.json 2>&1 || { tail -5 $O/pmc_sum_$i.json; exit 1; }
    cat $O/pmc_sum_$i.json
  done
  exit 0
fi
if [ "$CALL" = d ]; then  # how the input was written vs the tile pass's speed; the ID-compare experiment in the full suite order
  step write-state
  timeout -k 10 400 python -u tools/probes/write_state.py > $O/write_state.json 2> $O/write_state.err || { tail -20 $O/write_state.err; exit 1; }
  cat $O/write_state.json
  step verify-off-and-ring
  timeout -k 10 600 python -u -m pytest tests/test_gpu_verify_off.py tests/test_gpu_ring.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_voff.log 2>&1 || { tail -30 $O/pytest_voff.log; exit 1; }
  tail -1 $O/pytest_voff.log
  step e2e-fd
  timeout -k 10 400 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/bench_e2e_fd.json 2> $O/bench_e2e_fd.err || { tail -20 $O/bench_e2e_fd.err; exit 1; }
  cat $O/bench_e2e_fd.json
  timeout -k 10 400 python -u bench.py --e2e --fd --dev-cap 2 --steps 3 --warmup 1 > $O/bench_e2e_fd_cap2.json 2> $O/bench_e2e_fd_cap2.err || { tail -20 $O/bench_e2e_fd_cap2.err; exit 1; }
  cat $O/bench_e2e_fd_cap2.json
  step idc-suite
  SHOCKIDX_VARIANT=idc timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -v --timeout 300 --timeout-method thread -k "not 2gib_cap and not subset_50gib and not c5_80gib" > $O/pytest_idc.log 2>&1; echo "idc suite rc=$?"
  tail -3 $O/pytest_idc.log
  grep -E "FAILED|seed=" $O/pytest_idc.log | head -5
  exit 0
fi
if [ "$CALL" = e ]; then  # blocked tile order with batched line stores (SIDX_FQ_BLK) against the grid-stride order
  step parity-blk
  SHOCKIDX_VARIANT=blk timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not fasta and not 2gib_cap and not subset_50gib and not c5_80gib and not line" > $O/pytest_blk.log 2>&1 || { tail -30 $O/pytest_blk.log; exit 1; }
  tail -1 $O/pytest_blk.log
  step ab
  timeout -k 10 700 python -u tools/ab_inproc.py base blk blk1 --copies 4 --rounds 4 --per 5 --turn-warmup 20 --check-rows > $O/ab_fq.json 2> $O/ab_fq.err || { tail -20 $O/ab_fq.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ab_fq.json'));print({k:(v['k_med'],v['b_med'],v['count_ok']) for k,v in d['ab'].items()}, d['rows_agree'])"
  exit 0
fi
if [ "$CALL" = f ]; then  # the FASTA pass with the FASTQ pass's store pattern (SIDX_FA_BLK) against the grid-stride order
  step parity-fablk
  SHOCKIDX_VARIANT=fablk timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fasta_tiles.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not 2gib_cap and not subset_50gib and not c5_80gib and not fastq_gen and not create_fd" > $O/pytest_fablk.log 2>&1 || { tail -30 $O/pytest_fablk.log; exit 1; }
  tail -1 $O/pytest_fablk.log
  step ab
  timeout -k 10 700 python -u tools/ab_inproc.py base fablk --fmt fasta --copies 4 --rounds 4 --per 5 --turn-warmup 20 --check-rows > $O/ab_fa.json 2> $O/ab_fa.err || { tail -20 $O/ab_fa.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ab_fa.json'));print({k:(v['k_med'],v['b_med'],v['count_ok']) for k,v in d['ab'].items()}, d['rows_agree'])"
  exit 0
fi
if [ "$CALL" = g ]; then  # the tile passes timed by their dispatch packets: parity spot-check and the driver's line
  step parity
  timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_gpu_fasta_tiles.py tests/test_gpu_line.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
  step driver-bench
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { tail -20 $O/bench_driver_cmd.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_driver_cmd.json'));print(d['ms_per_step'],d['index_kernel_ms'],d['roofline']['frac'],d['build'],d['box_floor']['kernel_over_floor'])"
  step copies
  timeout -k 10 300 python -u tools/probes/copy_pmc.py --copies 4 --per 4 > $O/copies.json 2> $O/copies.err || { tail -20 $O/copies.err; exit 1; }
  cat $O/copies.json
  exit 0
fi
if [ "$CALL" = h ]; then  # the write-state probe again (needs a box where the generator's buffer is the slow one)
  step write-state
  timeout -k 10 400 python -u tools/probes/write_state.py > $O/write_state.json 2> $O/write_state.err || { tail -20 $O/write_state.err; exit 1; }
  cat $O/write_state.json
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

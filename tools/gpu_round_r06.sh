#!/bin/bash
# Round-6 measurement pass (run on the GPU box; outputs under gpurun_out/r06m/, copied to profiles/r06/):
#  PART=A: the -m gpu suite (SHOCKIDX_VERIFY on, tests/conftest.py) and smoke(); FASTQ (C2) / FASTA
#          (C3) / line: bench line, rocprofv3 kernel trace of the same command, FETCH_SIZE and
#          WRITE_SIZE in separate --pmc passes summarised for the tile kernel and the placement
#          kernel, SQ passes for the FASTQ / FASTA tile kernels; the driver's own bench command last
#  PART=B: end to end (pinned body; page-cached node file: build_fd, create, create with a 1 GiB
#          trim between builds), C4 subset with the gather's PMC, chunkrecord, the download filters,
#          the driver's 2-rank launch line with both ranks on the one GPU (host summary exchange)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r06m; mkdir -p $O
TAG=r06
step() { echo "== $* ($(date +%T))"; }
PART=${PART:-A}
if [ "$PART" = F ]; then  # the FASTQ line alone (kernel sources changed after part A): trace, PMC, default bench
  rm -rf $O/prof_kt_fastq $O/prof_fetch_fastq $O/prof_write_fastq
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_kt_fastq -o kt --output-format csv -- python3 $R/bench.py --fmt fastq > $O/bench_kt_fastq.json 2> $O/bench_kt_fastq.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_fastq -o pmc --output-format csv -- python3 $R/bench.py --fmt fastq --steps 3 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/bench_fetch_fastq.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_fastq -o pmc --output-format csv -- python3 $R/bench.py --fmt fastq --steps 3 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/bench_write_fastq.err || exit 1
  python tools/pmc_summary.py $O/prof_kt_fastq $O/prof_fetch_fastq $O/prof_write_fastq $O/pmc_${TAG}_fastq.json fastq > $O/pmc_${TAG}_fastq.log 2>&1 || exit 1
  PMC_KERNEL=k_fq_place python tools/pmc_summary.py $O/prof_kt_fastq $O/prof_fetch_fastq $O/prof_write_fastq $O/pmc_${TAG}_k_fq_place.json fastq > $O/pmc_${TAG}_k_fq_place.log 2>&1 || exit 1
  mkdir -p profiles/$TAG && cp $O/pmc_${TAG}_fastq.json profiles/$TAG/pmc_fastq.json
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit 1
  cat $O/bench_driver_cmd.json
  [ -n "$THEN_B" ] || exit 0
  PART=B
fi
if [ "$PART" = A ]; then
step suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
for FMT in fastq fasta; do
  step $FMT
  PK=$([ $FMT = fastq ] && echo k_fq_place || echo k_fa_place)
  rm -rf $O/prof_kt_$FMT $O/prof_fetch_$FMT $O/prof_write_$FMT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_kt_$FMT -o kt --output-format csv -- python3 $R/bench.py --fmt $FMT > $O/bench_kt_$FMT.json 2> $O/bench_kt_$FMT.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_$FMT -o pmc --output-format csv -- python3 $R/bench.py --fmt $FMT --steps 3 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/bench_fetch_$FMT.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_$FMT -o pmc --output-format csv -- python3 $R/bench.py --fmt $FMT --steps 3 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/bench_write_$FMT.err || exit 1
  python tools/pmc_summary.py $O/prof_kt_$FMT $O/prof_fetch_$FMT $O/prof_write_$FMT $O/pmc_${TAG}_$FMT.json $FMT > $O/pmc_${TAG}_$FMT.log 2>&1 || exit 1
  PMC_KERNEL=$PK python tools/pmc_summary.py $O/prof_kt_$FMT $O/prof_fetch_$FMT $O/prof_write_$FMT $O/pmc_${TAG}_${PK}.json $FMT > $O/pmc_${TAG}_${PK}.log 2>&1 || exit 1
  head -c 400 $O/pmc_${TAG}_$FMT.log; echo
done
step line
rm -rf $O/prof_kt_line $O/prof_fetch_line $O/prof_write_line
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_kt_line -o kt --output-format csv -- python3 $R/bench.py --kind line --cpu-sec 0 > $O/bench_line.json 2> $O/bench_line.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_line -o pmc --output-format csv -- python3 $R/bench.py --kind line --steps 3 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/fetch_line.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_line -o pmc --output-format csv -- python3 $R/bench.py --kind line --steps 3 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/write_line.err || exit 1
for K in k_line_tiles k_line_place; do
  PMC_KERNEL=$K python tools/pmc_summary.py $O/prof_kt_line $O/prof_fetch_line $O/prof_write_line $O/pmc_${TAG}_$K.json fastq > $O/pmc_${TAG}_$K.log 2>&1 || exit 1
done
step sq
i=0
for fmt in fastq fasta; do
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES"; do
    i=$((i+1)); rm -rf $O/sq_${fmt}_$i
    timeout -s KILL 120 rocprofv3 --pmc $set -d $O/sq_${fmt}_$i -o pmc --output-format csv -- python3 $R/bench.py --fmt $fmt --steps 2 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2> $O/sq_${fmt}_$i.err || exit 1
  done
done
for f in fastq fasta; do for i in 1 2 3 4; do [ -d $O/sq_${f}_$i ] && KN=$([ $f = fastq ] && echo k_fq_tiles || echo k_fa_tiles) python tools/sq_table.py r06m/sq_${f}_$i; done; done > $O/sq_summary.txt 2>&1
step default
mkdir -p profiles/$TAG && cp $O/pmc_${TAG}_fastq.json profiles/$TAG/pmc_fastq.json && cp $O/pmc_${TAG}_fasta.json profiles/$TAG/pmc_fasta.json
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit 1
cat $O/bench_driver_cmd.json
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cat $O/bench_default.json
exit 0
fi
step e2e
timeout -k 10 400 python -u bench.py --e2e --pinned --steps 3 --warmup 1 > $O/bench_e2e_fastq_pinned.json 2> $O/bench_e2e_pinned.err || exit 1
timeout -k 10 400 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/bench_e2e_fastq_fd.json 2> $O/bench_e2e_fd.err || exit 1
timeout -k 10 400 python -u bench.py --e2e --fd --trim 1 --steps 3 --warmup 1 > $O/bench_e2e_fastq_fd_trim1.json 2> $O/bench_e2e_fd_trim1.err || exit 1
timeout -k 10 400 python -u bench.py --e2e --fd --dev-cap 2 --steps 3 --warmup 1 > $O/bench_e2e_fastq_fd_cap2.json 2> $O/bench_e2e_fd_cap2.err || exit 1
step subset
rm -rf $O/prof_kt_subset $O/prof_fetch_subset $O/prof_write_subset
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt_subset -o kt --output-format csv -- python3 $R/bench.py --subset --steps 5 --warmup 2 > $O/bench_subset.json 2> $O/bench_subset.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_subset -o pmc --output-format csv -- python3 $R/bench.py --subset --steps 2 --warmup 1 > /dev/null 2> $O/pmc_subset_fetch.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_subset -o pmc --output-format csv -- python3 $R/bench.py --subset --steps 2 --warmup 1 > /dev/null 2> $O/pmc_subset_write.err || exit 1
PMC_KERNEL=k_gather python tools/pmc_summary.py $O/prof_kt_subset $O/prof_fetch_subset $O/prof_write_subset $O/pmc_${TAG}_gather.json fastq 536657358 > $O/pmc_${TAG}_gather.log 2>&1 || exit 1
step chunkrecord
for f in fastq fasta; do
  rm -rf $O/chunk_kt_$f
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/chunk_kt_$f -o run -- python3 bench.py --kind chunkrecord --fmt $f --steps 5 --warmup 1 --no-check > $O/bench_chunk_$f.json 2> $O/bench_chunk_$f.err || exit 1
done
step filters
for c in "fastq fq2fa" "fastq anonymize" "fasta anonymize"; do
  set -- $c
  rm -rf $O/filt_kt_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/filt_kt_$1_$2 -o run -- python3 bench.py --kind filter --fmt $1 --filter $2 --steps 5 --warmup 1 > $O/bench_filter_$1_$2.json 2> $O/bench_filter_$1_$2.err || exit 1
done
step rehearsal
SHOCKIDX_BENCH_DEVICE=0 SHOCKIDX_BENCH_EXCHANGE=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_rehearsal_2ranks_1gpu.json 2> $O/bench_rehearsal.err || exit 1
exit 0

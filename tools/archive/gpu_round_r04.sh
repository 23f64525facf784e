#!/bin/bash
# Round-4 measurement pass (run on the GPU box; outputs under gpurun_out/, copied to profiles/r04/):
#  - the -m gpu suite and smoke()
#  - FASTQ (C2) / FASTA (C3) / line: bench line, rocprofv3 kernel trace of the same command, the two
#    HBM PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) summarised for the dominant tile kernel
#    and the placement kernel, SQ counter passes for the FASTQ / FASTA tile kernels
#  - end to end: pinned body (slab pipeline), page-cached node file (build_fd / create pipeline)
#  - C4 subset with the gather's PMC, chunkrecord, the download filters with their writers' PMC
#  - the default `python bench.py` line last, with this round's PMC summary in place
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
TAG=r04
step() { echo "== $* ($(date +%T))"; }
PART=${PART:-A}
if [ "$PART" = A ]; then
step suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
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
bash tools/gpu_sq.sh > $O/sq.log 2>&1 || exit 1
step default
mkdir -p profiles/$TAG && cp $O/pmc_${TAG}_fastq.json profiles/$TAG/pmc_fastq.json && cp $O/pmc_${TAG}_fasta.json profiles/$TAG/pmc_fasta.json
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cat $O/bench_default.json
exit 0
fi
step e2e
timeout -k 10 400 python -u bench.py --e2e --pinned --steps 3 --warmup 1 > $O/bench_e2e_fastq_pinned.json 2> $O/bench_e2e_pinned.err || exit 1
timeout -k 10 400 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/bench_e2e_fastq_fd.json 2> $O/bench_e2e_fd.err || exit 1
step subset
rm -rf $O/prof_kt_subset $O/prof_fetch_subset $O/prof_write_subset
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt_subset -o kt --output-format csv -- python3 $R/bench.py --subset --steps 5 --warmup 2 > $O/bench_subset.json 2> $O/bench_subset.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_subset -o pmc --output-format csv -- python3 $R/bench.py --subset --steps 2 --warmup 1 > /dev/null 2> $O/pmc_subset_fetch.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_subset -o pmc --output-format csv -- python3 $R/bench.py --subset --steps 2 --warmup 1 > /dev/null 2> $O/pmc_subset_write.err || exit 1
PMC_KERNEL=k_gather python tools/pmc_summary.py $O/prof_kt_subset $O/prof_fetch_subset $O/prof_write_subset $O/pmc_${TAG}_gather.json fastq 536657358 > $O/pmc_${TAG}_gather.log 2>&1 || exit 1
step chunkrecord
for f in fastq fasta; do
  rm -rf $O/chunk_kt_$f $O/chunk_fetch_$f $O/chunk_write_$f
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/chunk_kt_$f -o run -- python3 bench.py --kind chunkrecord --fmt $f --steps 5 --warmup 1 --no-check > $O/bench_chunk_$f.json 2> $O/bench_chunk_$f.err || exit 1
done
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/chunk_fetch_fastq -o pmc --output-format csv -- python3 bench.py --kind chunkrecord --fmt fastq --steps 2 --warmup 1 --no-check > /dev/null 2> $O/chunk_fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/chunk_write_fastq -o pmc --output-format csv -- python3 bench.py --kind chunkrecord --fmt fastq --steps 2 --warmup 1 --no-check > /dev/null 2> $O/chunk_write.err || exit 1
PMC_KERNEL=k_cr_verify python tools/pmc_summary.py $O/chunk_kt_fastq $O/chunk_fetch_fastq $O/chunk_write_fastq $O/pmc_${TAG}_k_cr_verify.json fastq > $O/pmc_${TAG}_k_cr_verify.log 2>&1 || exit 1
step filters
for c in "fastq fq2fa k_fq_write" "fastq anonymize k_fq_write" "fasta anonymize k_fa_anon_write"; do
  set -- $c
  rm -rf $O/filt_kt_$1_$2 $O/filt_fetch_$1_$2 $O/filt_write_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/filt_kt_$1_$2 -o run -- python3 bench.py --kind filter --fmt $1 --filter $2 --steps 5 --warmup 1 > $O/bench_filter_$1_$2.json 2> $O/bench_filter_$1_$2.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/filt_fetch_$1_$2 -o pmc --output-format csv -- python3 bench.py --kind filter --fmt $1 --filter $2 --steps 2 --warmup 1 > /dev/null 2> $O/filt_fetch_$1_$2.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/filt_write_$1_$2 -o pmc --output-format csv -- python3 bench.py --kind filter --fmt $1 --filter $2 --steps 2 --warmup 1 > /dev/null 2> $O/filt_write_$1_$2.err || exit 1
  PMC_KERNEL=$3 python tools/pmc_summary.py $O/filt_kt_$1_$2 $O/filt_fetch_$1_$2 $O/filt_write_$1_$2 $O/pmc_${TAG}_filter_$1_$2.json $1 > $O/pmc_${TAG}_filter_$1_$2.log 2>&1 || exit 1
done
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
exit 0

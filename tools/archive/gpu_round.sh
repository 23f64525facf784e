#!/bin/bash
# Round measurement (TAG=r03 ...): the -m gpu suite; FASTQ (C2) and FASTA (C3) bench lines with kernel
# traces and HBM PMC passes; line; the end-to-end lines (pinned slab pipeline, page-cached fd);
# the C4 subset line with k_gather PMC; chunkrecord and download-filter kernel traces; smoke.  Outputs: gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r03} FMT=fastq bash tools/gpu_measure.sh || exit 1
echo "fastq done"; tail -1 $O/pytest_gpu.log
SKIP_TESTS=1 TAG=${TAG:-r03} FMT=fasta bash tools/gpu_measure.sh || exit 1
echo "fasta done"
rm -rf $O/prof_kt_line
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_kt_line -o kt --output-format csv -- python3 $R/bench.py --kind line --cpu-sec 0 > $O/bench_line.json 2> $O/bench_line.err || exit 1
timeout -k 10 400 python -u bench.py --e2e --pinned --steps 3 --warmup 1 > $O/bench_e2e_fastq_pinned.json 2> $O/bench_e2e_pinned.err || exit 1
timeout -k 10 400 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/bench_e2e_fastq_fd.json 2> $O/bench_e2e_fd.err || exit 1
echo "e2e done"
rm -rf $O/prof_kt_subset $O/prof_fetch_subset $O/prof_write_subset
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt_subset -o kt --output-format csv -- python3 $R/bench.py --subset --steps 5 --warmup 2 > $O/bench_subset.json 2> $O/bench_subset.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_subset -o pmc --output-format csv -- python3 $R/bench.py --subset --steps 2 --warmup 1 > /dev/null 2> $O/pmc_subset_fetch.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_subset -o pmc --output-format csv -- python3 $R/bench.py --subset --steps 2 --warmup 1 > /dev/null 2> $O/pmc_subset_write.err || exit 1
PMC_KERNEL=k_gather python tools/pmc_summary.py $O/prof_kt_subset $O/prof_fetch_subset $O/prof_write_subset $O/pmc_${TAG:-r03}_gather.json fastq 536657358 > $O/pmc_${TAG:-r03}_gather.log 2>&1
echo "subset done"
for f in fastq fasta; do
  rm -rf $O/chunk_kt_$f
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/chunk_kt_$f -o run -- python3 bench.py --kind chunkrecord --fmt $f --steps 5 --warmup 1 --no-check > $O/bench_chunk_$f.json 2> $O/bench_chunk_$f.err || exit 1
done
for c in "fastq fq2fa" "fastq anonymize" "fasta anonymize"; do
  set -- $c
  rm -rf $O/filt_kt_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/filt_kt_$1_$2 -o run -- python3 bench.py --kind filter --fmt $1 --filter $2 --steps 5 --warmup 1 > $O/bench_filter_$1_$2.json 2> $O/bench_filter_$1_$2.err || exit 1
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
exit 0

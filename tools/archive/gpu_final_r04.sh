#!/bin/bash
# Round 4 closing pass on the final kernel sources (outputs under gpurun_out/final/, copied to
# profiles/r04/): the GPU suite; FASTQ / FASTA bench lines with their kernel traces and the two
# HBM PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) -> pmc_<fmt>.json, which bench.py takes
# for roofline.traffic while the sources match; line, chunkrecord, SAM and FASTA-anonymize
# traces; a 2-rank rehearsal of the multi-GPU bench on one device; the default bench line; smoke.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/final; mkdir -p $O
step() { echo "== $* ($(date +%T))"; }
if [ "${SKIP_SUITE:-0}" != 1 ]; then
step suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
for FMT in fastq fasta; do
  step $FMT
  rm -rf $O/kt_$FMT $O/fetch_$FMT $O/write_$FMT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$FMT -o kt --output-format csv -- python3 $R/bench.py --fmt $FMT > $O/bench_$FMT.json 2> $O/bench_$FMT.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$FMT -o pmc --output-format csv -- python3 $R/bench.py --fmt $FMT --steps 3 --warmup 1 --cpu-sec 0 --no-check --no-floor > /dev/null 2> $O/fetch_$FMT.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write_$FMT -o pmc --output-format csv -- python3 $R/bench.py --fmt $FMT --steps 3 --warmup 1 --cpu-sec 0 --no-check --no-floor > /dev/null 2> $O/write_$FMT.err || exit 1
  python tools/pmc_summary.py $O/kt_$FMT $O/fetch_$FMT $O/write_$FMT $O/pmc_$FMT.json $FMT > $O/pmc_$FMT.log 2>&1 || exit 1
done
step line
rm -rf $O/kt_line
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_line -o kt --output-format csv -- python3 $R/bench.py --kind line --cpu-sec 0 > $O/bench_line.json 2> $O/bench_line.err || exit 1
step chunkrecord
rm -rf $O/kt_chunk
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_chunk -o kt --output-format csv -- python3 $R/bench.py --kind chunkrecord --fmt fastq --steps 5 --warmup 2 > $O/bench_chunk_fastq.json 2> $O/bench_chunk_fastq.err || exit 1
step sam
rm -rf $O/kt_sam
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_sam -o kt --output-format csv -- python3 $R/tools/sam_bench.py > $O/bench_sam.json 2> $O/bench_sam.err || exit 1
step anonymize
rm -rf $O/kt_anon
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_anon -o kt --output-format csv -- python3 $R/bench.py --kind filter --fmt fasta --filter anonymize --steps 5 --warmup 1 > $O/bench_filter_fasta_anonymize.json 2> $O/bench_filter_fasta_anonymize.err || exit 1
step rehearsal
SHOCKIDX_BENCH_DEVICE=0 SHOCKIDX_BENCH_EXCHANGE=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_rehearsal_2ranks_1gpu.json 2> $O/bench_rehearsal.err || { tail -20 $O/bench_rehearsal.err; exit 1; }
step default
mkdir -p profiles/r04 && cp $O/pmc_fastq.json profiles/r04/pmc_fastq.json && cp $O/pmc_fasta.json profiles/r04/pmc_fasta.json
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cat $O/bench_default.json
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
exit 0

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 200 python -u bench.py --fmt fastq --steps 20 --warmup 3 --cpu-sec 0 > $O/b0_fastq.json 2> $O/b0_fastq.err || exit 1
timeout -k 10 200 python -u bench.py --fmt fasta --steps 20 --warmup 3 --cpu-sec 0 > $O/b0_fasta.json 2> $O/b0_fasta.err || exit 1
bash tools/gpu_sq.sh > $O/sq.log 2>&1 || exit 1
rm -rf $O/kt0; timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt0 -o kt --output-format csv -- python3 bench.py --fmt fastq --steps 20 --warmup 3 --cpu-sec 0 > $O/kt0.json 2>$O/kt0.err || exit 1
echo done

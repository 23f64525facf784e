#!/bin/bash
# Round 4, late: the tile body's four LDS-DMA pieces under one M0 (m0once variant) -- parity of
# the FASTQ / FASTA / line builds with it (bench row checks), then A/B against the current build.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
for k in "--fmt fastq" "--fmt fasta" "--kind line"; do
  SHOCKIDX_VARIANT=m0once timeout -k 10 300 python bench.py $k --steps 5 --warmup 3 --cpu-sec 0 --no-floor > $O/m0once_check.json 2> $O/m0once_check.err || { cat $O/m0once_check.err | tail -5; exit 1; }
  python -c "import json;d=json.load(open('$O/m0once_check.json'));print('$k', d.get('parity', d.get('parity_ok')), d.get('index_kernel_ms'))"
done
VARS="base m0once" ROUNDS=3 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fastq.txt $O/ab_m0once_fastq.txt
FMT=fasta VARS="base m0once" ROUNDS=2 bash tools/gpu_ab.sh || exit 1
cp $O/ab_fasta.txt $O/ab_m0once_fasta.txt
exit 0

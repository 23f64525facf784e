#!/bin/bash
# Page-cache DMA chunking: chunk size / chunks kept pinned, against the pread staging path.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
run() { timeout -k 10 400 python -u bench.py --e2e --fd --steps 3 --warmup 1 > $O/e2e_$1.json 2> $O/e2e_$1.err && python -c "import json;d=json.load(open('$O/e2e_$1.json'));print('$1', d['value'], d['create_gib_s'], d['timings_ms']['h2d_ms'])"; }
for r in 1 2; do
  SHOCKIDX_NO_MMAP_DMA=1 run pread_$r || exit 1
  SHOCKIDX_MMAP_CHUNK_MIB=1024 SHOCKIDX_MMAP_PINNED=64 run m1024_all_$r || exit 1
  SHOCKIDX_MMAP_CHUNK_MIB=256 SHOCKIDX_MMAP_PINNED=64 run m256_all_$r || exit 1
  SHOCKIDX_MMAP_CHUNK_MIB=64 SHOCKIDX_MMAP_PINNED=1024 run m64_all_$r || exit 1
done
exit 0

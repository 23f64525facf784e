#!/bin/bash
# Round 4, late: chunkrecord verify (run starts from the class words) and the SAM tile pass --
# their GPU tests, the chunkrecord A/B against the previous verify kernel, the SAM build timing,
# then the record / line bench lines with the box's streaming floor.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sam.py tests/test_gpu_chunk.py -x -q --timeout 200 --timeout-method thread > $O/r04c_tests.log 2>&1 || { tail -30 $O/r04c_tests.log; exit 1; }
tail -2 $O/r04c_tests.log
timeout -k 10 300 python -u tools/sam_bench.py > $O/sam_bench.json 2> $O/sam_bench.err || { tail -5 $O/sam_bench.err; exit 1; }
cat $O/sam_bench.json
KIND=chunkrecord VARS="base crold" ROUNDS=2 bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 python bench.py --cpu-sec 0 > $O/floor_fastq.json 2> $O/floor_fastq.err || exit 1
timeout -k 10 300 python bench.py --kind line --cpu-sec 0 > $O/floor_line.json 2> $O/floor_line.err || exit 1
cat $O/floor_fastq.json $O/floor_line.json
exit 0

#!/bin/bash
# After two minutes of GPU load (the suite): is the slow k_fq_tiles state the placement of the
# buffers the tile pass writes?  The default bench, then with the stage workspace contiguous
# (SHOCKIDX_CONTIG_WS=2), then with the input in ordinary memory (SHOCKIDX_NO_CONTIG).
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/thermal2; mkdir -p $O
b() { timeout -k 10 300 python bench.py --cpu-sec 0 > $O/bench_$1.json 2> $O/bench_$1.err && python -c "import json;d=json.load(open('$O/bench_$1.json'));print('$1', d['index_kernel_ms'], d['build']['kernel_ms'], d['box_floor']['ms'])"; }
b fresh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b after_suite || exit 1
SHOCKIDX_CONTIG_WS=2 b contig_stage || exit 1
SHOCKIDX_NO_CONTIG=1 b input_plain || exit 1
b again || exit 1
exit 0

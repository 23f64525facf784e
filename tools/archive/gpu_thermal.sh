#!/bin/bash
# Is the slow state of k_fq_tiles brought on by sustained load?  The default bench on a fresh
# process first, then after the GPU suite (two minutes of load), then after a minute idle.
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/thermal; mkdir -p $O
b() { timeout -k 10 300 python bench.py --cpu-sec 0 > $O/bench_$1.json 2> $O/bench_$1.err && python -c "import json;d=json.load(open('$O/bench_$1.json'));print('$1', d['index_kernel_ms'], d['build']['kernel_ms'], d['box_floor']['ms'])"; }
b fresh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b after_suite || exit 1
sleep 60
b after_idle || exit 1
exit 0

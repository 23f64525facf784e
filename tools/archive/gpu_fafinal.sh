#!/bin/bash
# FASTA anonymize after the writer's 2 KiB steps: every filter GPU test, then the filter's bench
# under a kernel trace and the writer's HBM bytes (FETCH_SIZE, WRITE_SIZE passes).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/fafinal; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_filter.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --kind filter --fmt fasta --filter anonymize --steps 5 --warmup 1 > $O/bench_filter_fasta_anonymize.json 2> $O/bench.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- python3 bench.py --kind filter --fmt fasta --filter anonymize --steps 2 --warmup 1 > /dev/null 2> $O/fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv -- python3 bench.py --kind filter --fmt fasta --filter anonymize --steps 2 --warmup 1 > /dev/null 2> $O/write.err || exit 1
PMC_KERNEL=k_fa_anon_write python tools/pmc_summary.py $O/kt $O/fetch $O/write $O/pmc_filter_fasta_anonymize.json fasta > $O/pmc.log 2>&1 || exit 1
cat $O/bench_filter_fasta_anonymize.json
exit 0

#!/bin/bash
# FASTA tile pass: parity, bench, kernel stats, HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
TAG=${TAG:-fa}
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_fasta_tiles.py tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q \
  --timeout 300 --timeout-method thread -k "${TESTK:-fasta or tiny or fixture or kat or generated or huge}" > $O/${TAG}_pytest.log 2>&1 \
  || { tail -30 $O/${TAG}_pytest.log; exit 1; }
echo "pytest: $(tail -1 $O/${TAG}_pytest.log)"
fi
timeout -k 10 300 python bench.py --fmt fasta --steps 20 --cpu-sec 0 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
rm -rf $O/${TAG}_kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_kt -o run -- python3 bench.py --fmt fasta --steps 20 --cpu-sec 0 > /dev/null 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/${TAG}_$c
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${TAG}_$c -o pmc --output-format csv -- python3 bench.py --fmt fasta --steps 3 --warmup 1 --cpu-sec 0 --no-check > /dev/null 2>&1 || exit 1
done
python3 tools/pmc_summary.py $O/${TAG}_kt $O/${TAG}_FETCH_SIZE $O/${TAG}_WRITE_SIZE $O/${TAG}_pmc.json fasta $((10 << 30))

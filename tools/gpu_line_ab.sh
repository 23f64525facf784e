set -o pipefail
O=$(pwd)/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_line.py -x -q --timeout 120 --timeout-method thread > $O/lab_pytest.log 2>&1 || { tail -30 $O/lab_pytest.log; exit 1; }
tail -1 $O/lab_pytest.log
for v in ${VARS:-default lw8 lw9 default}; do
  if [ $v = default ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
  timeout -k 10 200 python bench.py --kind line --steps 20 --warmup 3 > $O/lab_$v.json 2>&1 || { tail $O/lab_$v.json; exit 1; }
  python -c "import json; d=json.load(open('$O/lab_$v.json')); print('$v', d['ms_per_step'], d['index_kernel_ms'], d['build']['kernel_ms'], d['parity_ok'])"
done

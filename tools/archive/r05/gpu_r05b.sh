#!/bin/bash
# round 5: the whole GPU suite (it also brings the box into the state the driver's bench sees
# after its own GPUTEST), then an interleaved A/B of the FASTQ tile-pass variants
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
(rocm-smi --showclocks --showtemp --showpower 2>&1 | head -40) > $O/smi_before.txt || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
(rocm-smi --showclocks --showtemp --showpower 2>&1 | head -40) > $O/smi_after_suite.txt || true
for i in 1 2; do
  for v in ring0 base cw32 cw16 r0cw32 t8k t8kdb; do
    if [ $v = base ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
    timeout -k 10 120 python bench.py --cpu-sec 0 --warmup 30 --steps 20 --no-floor > $O/ab_${v}_$i.json 2>&1 || exit $?
  done
done
unset SHOCKIDX_VARIANT
(rocm-smi --showclocks --showtemp --showpower 2>&1 | head -40) > $O/smi_after_ab.txt || true

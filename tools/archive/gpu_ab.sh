#!/bin/bash
# A/B of libshockidx variants (shock_amd/variants/libshockidx_<V>.so) on the default FASTQ bench:
# interleaved runs, one JSON line each, kernel ms summarised at the end.  VARS="base v1 v2" ROUNDS=2
# KIND=record|line|chunkrecord|filter (FILTER=fq2fa|anonymize)
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
FMT=${FMT:-fastq}
: > $O/ab_$FMT.txt
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARS:-base}; do
    if [ "$v" = base ]; then unset SHOCKIDX_VARIANT; else export SHOCKIDX_VARIANT=$v; fi
    timeout -k 10 240 python -u bench.py --kind ${KIND:-record} --filter ${FILTER:-fq2fa} --fmt $FMT --steps 20 --warmup 3 --cpu-sec 0 --no-check > $O/ab_${FMT}_$v.json 2> $O/ab_${FMT}_$v.err
    rc=$?
    # ablation variants (abl*) skip work, so their tables are wrong by design: keep the timing
    if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ "${v#abl}" = "$v" ]; }; then echo "variant $v failed ($rc)"; tail -5 $O/ab_${FMT}_$v.err; exit 1; fi
    python -c "import json,sys;d=json.load(open('$O/ab_${FMT}_$v.json'));print('$v', d.get('index_kernel_ms', d.get('kernel_ms')), d.get('build', {}).get('kernel_ms'), d['ms_per_step'])" >> $O/ab_$FMT.txt
  done
done
unset SHOCKIDX_VARIANT
cat $O/ab_$FMT.txt

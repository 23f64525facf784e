#!/bin/bash
# round 5: which FASTQ start-array layout breaks fresh-context host builds (probe), verify off
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
SHOCKIDX_VERIFY=0 timeout -k 10 120 python -u tools/probes/fq_layout_probe.py base ilpk0 il0 > $O/probe_noverify2.txt 2>&1 || exit $?

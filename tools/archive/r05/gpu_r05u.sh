#!/bin/bash
# round 5: does the way the node body was written (kernel vs copy engine) set the tile pass's speed?
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 400 python -u tools/probes/placement_writer.py > $O/placement_writer.json 2> $O/placement_writer.err || exit $?

#!/bin/bash
# Round-6 late A/B call: FASTA batch sizes, then the rotate-by-permute mask assembly on FASTQ and
# FASTA (tools/probes/fa_rr_variants.py, rotperm_variant.py); one process per table.
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 400 python -u tools/ab_inproc.py base farr16 farr24 farr48 farr64 --fmt fasta --copies 3 --check-rows > $O/ab_fa_batch.json 2> $O/ab1.err || { tail -5 $O/ab1.err; exit 1; }
cat $O/ab_fa_batch.json
timeout -k 10 300 python -u tools/ab_inproc.py base rotperm --fmt fastq --copies 3 --check-rows > $O/ab_fq_rotperm.json 2> $O/ab2.err || { tail -5 $O/ab2.err; exit 1; }
cat $O/ab_fq_rotperm.json
timeout -k 10 300 python -u tools/ab_inproc.py base rotperm --fmt fasta --copies 3 --check-rows > $O/ab_fa_rotperm.json 2> $O/ab3.err || { tail -5 $O/ab3.err; exit 1; }
cat $O/ab_fa_rotperm.json

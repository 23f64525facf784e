set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/repeat_check.py fastq 1 40 auto > gpurun_out/rep1.log 2>&1 && \
timeout -k 10 300 python tools/repeat_check.py fastq 1 40 fastq >> gpurun_out/rep1.log 2>&1 && \
timeout -k 10 300 python tools/repeat_check.py fastq 10 6 auto >> gpurun_out/rep1.log 2>&1 && \
timeout -k 10 300 python tools/repeat_check.py fasta 1 20 auto >> gpurun_out/rep1.log 2>&1

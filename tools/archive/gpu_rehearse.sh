#!/bin/bash
# multi-rank rehearsal on a one-GPU box: 2 ranks on device 0 over the host summary exchange
# (RCCL needs distinct devices), the driver's torch.distributed.run launch line otherwise
set -o pipefail
O=$(pwd)/gpurun_out; mkdir -p $O
SHOCKIDX_BENCH_DEVICE=0 SHOCKIDX_BENCH_EXCHANGE=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_rehearsal_2ranks_1gpu.json 2> $O/bench_rehearsal_2ranks_1gpu.err || { tail -20 $O/bench_rehearsal_2ranks_1gpu.err; exit 1; }
cat $O/bench_rehearsal_2ranks_1gpu.json

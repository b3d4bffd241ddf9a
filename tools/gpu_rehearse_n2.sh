#!/bin/bash
# Rehearse the bench's N>1 path on a one-GPU box: two ranks share cuda:0
# (OGS_BENCH_SHARE_DEVICE=1, gloo for the per-rank records). Checks that every
# config's sharded run completes and prints one line; the numbers are not
# scaling numbers (both ranks time-share one GPU).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
export OGS_BENCH_SHARE_DEVICE=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 \
  > gpurun_out/rehearse_n2.log 2>&1
rc=$?
echo "rehearse_n2 rc=$rc"; grep '^{' gpurun_out/rehearse_n2.log | cut -c1-600
tail -5 gpurun_out/rehearse_n2.log | cut -c1-300
exit $rc

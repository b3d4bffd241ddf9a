#!/bin/bash
# Round 4: C3 stream geometry sweep (threads per workgroup x workgroups per
# unit) on the N = 8 / 4 / 2 rank shards and the whole build, in-process A/B.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
V="frontier_block=256,frontier_parts=1 frontier_block=256,frontier_parts=2 frontier_block=256,frontier_parts=4 frontier_block=512,frontier_parts=1 frontier_block=512,frontier_parts=2 frontier_block=1024,frontier_parts=1 frontier_block=1024,frontier_parts=2"
for r in 0/8 0/4 0/2; do
  echo "=== shard $r"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 3 --as-rank $r $V > gpurun_out/r04_geom_${r/\//_}.log 2>&1 || { tail -30 gpurun_out/r04_geom_${r/\//_}.log; exit 1; }
  grep '^{' gpurun_out/r04_geom_${r/\//_}.log
done
echo "=== full"
timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 3 frontier_block=256,frontier_parts=1 frontier_block=256,frontier_parts=2 frontier_block=512,frontier_parts=1 frontier_block=512,frontier_parts=2 > gpurun_out/r04_geom_full.log 2>&1 || { tail -30 gpurun_out/r04_geom_full.log; exit 1; }
grep '^{' gpurun_out/r04_geom_full.log

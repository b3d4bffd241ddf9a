#!/bin/bash
# Round 4, first box: C3 shard projection (N = 2/4/8 ranks, each alone),
# the shard-XOR parity test, and the frontier_o8 A/B (in-process, interleaved).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_size.py -k "rank_shards" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_shard_test.log 2>&1 || { tail -30 gpurun_out/r04_shard_test.log; exit 1; }
tail -3 gpurun_out/r04_shard_test.log
timeout -k 10 400 python -u bench.py --config c3 --steps 20 --no-cpu-baseline --no-extras > gpurun_out/r04_c3_proj.json 2> gpurun_out/r04_c3_proj.log || { tail -30 gpurun_out/r04_c3_proj.log; exit 1; }
cat gpurun_out/r04_c3_proj.log
timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 5 frontier_o8=0 frontier_o8=1 > gpurun_out/r04_o8_ab.log 2>&1 || { tail -30 gpurun_out/r04_o8_ab.log; exit 1; }
cat gpurun_out/r04_o8_ab.log
timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 5 --as-rank 0/8 frontier_o8=0 frontier_o8=1 route_stream=1 > gpurun_out/r04_o8_ab_r8.log 2>&1 || { tail -30 gpurun_out/r04_o8_ab_r8.log; exit 1; }
cat gpurun_out/r04_o8_ab_r8.log

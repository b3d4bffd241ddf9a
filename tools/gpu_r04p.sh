#!/bin/bash
# One-launch LDS SPF + stream (route_stream 5): parity, A/B over shards.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "route_stream" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04p_par.log 2>&1 || { tail -40 gpurun_out/r04p_par.log; exit 1; }
tail -2 gpurun_out/r04p_par.log
for r in 0/8 0/4 0/2 0/1; do
  echo "=== A/B $r"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 3 --as-rank $r frontier_block=512,frontier_parts=2,frontier_parts_wide=4 route_stream=4 route_stream=5 route_stream=5,lds_parts=2 route_stream=5,lds_parts=8 > gpurun_out/r04p_ab.log 2>&1 || { tail -30 gpurun_out/r04p_ab.log; exit 1; }
  grep '^{' gpurun_out/r04p_ab.log | cut -c1-150
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_size.py -k "every_source" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04p_c3.log 2>&1 || { tail -40 gpurun_out/r04p_c3.log; exit 1; }
tail -2 gpurun_out/r04p_c3.log

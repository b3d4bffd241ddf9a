#!/bin/bash
# One launch for all C3 width groups (ogs_spf_routes_groups): parity, A/B.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 0/8 0/4 0/2 0/1; do
  echo "=== A/B $r"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 3 --as-rank $r route_stream=5,c3groups=0 route_stream=5,lds_parts=2,c3groups=0 route_stream=5 route_stream=5,lds_parts=2 route_stream=5,lds_parts=3 route_stream=5,lds_parts=6 > gpurun_out/r04q_ab.log 2>&1 || { tail -30 gpurun_out/r04q_ab.log; exit 1; }
  grep '^{' gpurun_out/r04q_ab.log | cut -c1-150
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_size.py -k "every_source or shards" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04q_c3.log 2>&1 || { tail -40 gpurun_out/r04q_c3.log; exit 1; }
tail -2 gpurun_out/r04q_c3.log

#!/bin/bash
# One-launch form: store flavour / parts A/B at N=1 and N=8.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 0/1 0/8; do
  echo "=== A/B $r"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 4 --as-rank $r route_stream=5 route_stream=5,lds_parts=2 route_stream=5,route_store_nt=3 route_stream=5,lds_parts=2,route_store_nt=3 > gpurun_out/r04t_ab.log 2>&1 || { tail -30 gpurun_out/r04t_ab.log; exit 1; }
  grep '^{' gpurun_out/r04t_ab.log | cut -c1-150
done

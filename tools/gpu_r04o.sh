#!/bin/bash
# C3 shard timelines (kernel trace) for the LDS split and the fused kernel
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 0/8 0/1; do
  t=${r/\//_}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$t -o k -- python3 tools/c3_opt_ab.py --pairs 1 --steps 3 --warmup 1 --as-rank $r route_stream=5 > gpurun_out/tl_$t.log 2>&1 || { tail -20 gpurun_out/tl_$t.log; exit 1; }
  echo "=== $r"; grep '^{' gpurun_out/tl_$t.log | cut -c1-120
  python3 tools/trace_timeline.py $(find gpurun_out/tl_$t -name "*kernel_trace.csv" | head -1) 16
done

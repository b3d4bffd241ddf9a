#!/bin/bash
# Round 4: LDS-resident SPF + split stream (route_stream 4) parity and A/B.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "route_stream" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04h_par.log 2>&1 || { tail -40 gpurun_out/r04h_par.log; exit 1; }
tail -2 gpurun_out/r04h_par.log
g() { echo "frontier_block=$1,frontier_parts=$2,frontier_parts_wide=$3"; }
run() {
  local tag=$1 r=$2; shift 2
  local ar=""; [ "$r" != "-" ] && ar="--as-rank $r"
  echo "=== $tag"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 3 $ar "$@" > gpurun_out/r04h_$tag.log 2>&1 || { tail -30 gpurun_out/r04h_$tag.log; exit 1; }
  grep '^{' gpurun_out/r04h_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(f\"{d['variant']:70s} {d['median_ms']:.4f} ms frac {d['frac']:.3f} golden {d['golden']}\")"
}
run n8 0/8 "$(g 512 2 4)" route_stream=4 route_stream=4,frontier_parts=2,frontier_parts_wide=4 route_stream=4,frontier_parts=4,frontier_parts_wide=6 || exit 1
run n4 0/4 "$(g 512 1 2)" route_stream=4 route_stream=4,frontier_parts=2,frontier_parts_wide=4 || exit 1
run n2 0/2 "$(g 512 1 1)" route_stream=4 route_stream=4,frontier_parts=1,frontier_parts_wide=1 || exit 1
run n1 - "$(g 256 1 1)" route_stream=4 route_stream=4,frontier_parts=1,frontier_parts_wide=1 route_stream=4,frontier_parts=1,frontier_parts_wide=2 || exit 1

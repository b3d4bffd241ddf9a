#!/bin/bash
# Round 4: lane-walk chunk scan + pipelined edge loads + preloaded distances
# vs HEAD (lib=base), and the stream geometry per shard size.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
g() { echo "frontier_block=$1,frontier_parts=$2,frontier_parts_wide=$3"; }
run() {  # run <tag> <as-rank or -> variants...
  local tag=$1 r=$2; shift 2
  local ar=""; [ "$r" != "-" ] && ar="--as-rank $r"
  echo "=== $tag"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 3 $ar "$@" > gpurun_out/r04d_$tag.log 2>&1 || { tail -30 gpurun_out/r04d_$tag.log; exit 1; }
  grep '^{' gpurun_out/r04d_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(f\"{d['variant']:60s} {d['median_ms']:.4f} ms frac {d['frac']:.3f} golden {d['golden']}\")"
}
run n8 0/8 lib=base "$(g 256 1 1)" "$(g 512 1 1)" "$(g 1024 1 1)" "$(g 512 2 3)" "$(g 512 2 4)" "$(g 256 3 5)" "$(g 256 4 7)" "$(g 256 2 4)" || exit 1
run n4 0/4 lib=base "$(g 256 1 1)" "$(g 512 1 1)" "$(g 512 1 2)" "$(g 512 2 3)" "$(g 256 2 3)" "$(g 256 1 2)" "$(g 256 2 4)" || exit 1
run n2 0/2 lib=base "$(g 256 1 1)" "$(g 256 1 2)" "$(g 512 1 1)" "$(g 512 1 2)" "$(g 256 2 3)" || exit 1
run n1 - lib=base "$(g 256 1 1)" "$(g 256 1 2)" "$(g 256 1 3)" "$(g 512 1 1)" "$(g 512 1 2)" || exit 1

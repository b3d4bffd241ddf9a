#!/bin/bash
# Round 4: kernel trace of the route_stream 4 form (LDS SPF + split stream).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT"
for r in 0/8 0/1; do
  t=${r/\//_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$t -o k -- python3 tools/c3_opt_ab.py --pairs 1 --steps 5 --as-rank $r route_stream=4 > gpurun_out/prof_$t.log 2>&1 || { tail -20 gpurun_out/prof_$t.log; exit 1; }
  echo "=== $r"; grep '^{' gpurun_out/prof_$t.log
  grep -v "at::native\|rocclr_copy" gpurun_out/prof_$t/k_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done

#!/bin/bash
# Round 4: LDS SPF (batched reads, parallel image build): parity + trace.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "route_stream" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j_par.log 2>&1 || { tail -40 gpurun_out/r04j_par.log; exit 1; }
tail -2 gpurun_out/r04j_par.log
cd /tmp && cd "$GRAFT_REPO_ROOT"
for r in 0/8 0/1; do
  t=${r/\//_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$t -o k -- python3 tools/c3_opt_ab.py --pairs 1 --steps 5 --as-rank $r route_stream=4 > gpurun_out/prof_$t.log 2>&1 || { tail -20 gpurun_out/prof_$t.log; exit 1; }
  echo "=== $r"; grep '^{' gpurun_out/prof_$t.log
done

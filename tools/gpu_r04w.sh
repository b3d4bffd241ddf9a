#!/bin/bash
# Tail parts A/B at N=1 (and N=2), parity of the C3 build.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 0/1 0/2; do
  echo "=== $r"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 4 --as-rank $r lds_tail=1 lds_tail=0 lds_tail=1,lds_parts=2 lds_tail=0,lds_parts=4 > gpurun_out/r04w_ab.log 2>&1 || { tail -30 gpurun_out/r04w_ab.log; exit 1; }
  grep '^{' gpurun_out/r04w_ab.log | cut -c1-150
done

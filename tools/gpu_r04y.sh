#!/bin/bash
# Stream-order rotation: parity + A/B at N=8/4.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route_db_batch.py -k "route_stream or fabric" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04y_par.log 2>&1 || { tail -40 gpurun_out/r04y_par.log; exit 1; }
tail -1 gpurun_out/r04y_par.log
for r in 0/8 0/4; do
  echo "=== $r"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 4 --as-rank $r lds_rotate=1 lds_rotate=0 > gpurun_out/r04y_ab.log 2>&1 || { tail -30 gpurun_out/r04y_ab.log; exit 1; }
  grep '^{' gpurun_out/r04y_ab.log | cut -c1-150
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_size.py -k "shards" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04y_c3.log 2>&1 || { tail -40 gpurun_out/r04y_c3.log; exit 1; }
tail -1 gpurun_out/r04y_c3.log

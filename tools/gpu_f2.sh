#!/bin/bash
# f2 check: RouteDbBatch parity, then the full default bench line.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_route_db_batch.py tests/test_csr_patch.py -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/f2_tests.log 2>&1
rc=$?; tail -12 gpurun_out/f2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/f2_bench.log 2>&1
rc=$?; tail -2 gpurun_out/f2_bench.log | cut -c1-600; exit $rc

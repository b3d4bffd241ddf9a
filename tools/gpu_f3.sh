#!/bin/bash
# f1/f3 check: full GPU parity suite, then the C4 bench line.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/f3_tests.log 2>&1
rc=$?; tail -15 gpurun_out/f3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/f3_bench.log 2>&1
rc=$?; tail -3 gpurun_out/f3_bench.log | cut -c1-2500; exit $rc

#!/bin/bash
# f1 check: variant/route-update parity tests, then the C4 bench line.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/f1_tests.log 2>&1
rc=$?; tail -15 gpurun_out/f1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/f1_bench.log 2>&1
rc=$?; tail -3 gpurun_out/f1_bench.log | cut -c1-1500; exit $rc

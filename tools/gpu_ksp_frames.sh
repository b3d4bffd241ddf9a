#!/bin/bash
# KSP 8-byte frames: full GPU parity suite, then the C5 bench line.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/kf_tests.log 2>&1
rc=$?; tail -6 gpurun_out/kf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/kf_bench.log 2>&1
rc=$?; tail -1 gpurun_out/kf_bench.log | cut -c1-900; exit $rc

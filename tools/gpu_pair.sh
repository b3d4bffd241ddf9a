#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "pair or c2 or wave or grid" > gpurun_out/pair_tests.log 2>&1; rc=$?; tail -15 gpurun_out/pair_tests.log; [ $rc -eq 0 ] || exit $rc
OPTS="6/4" timeout -k 10 300 python -u tools/ab_wave_opt.py > gpurun_out/ab_pair.log 2>&1; rc=$?; cat gpurun_out/ab_pair.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1; rc=$?; tail -c 1500 gpurun_out/bench_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config g1 --no-cpu-baseline > gpurun_out/bench_g1.log 2>&1; rc=$?; tail -c 1500 gpurun_out/bench_g1.log; exit $rc

#!/bin/bash
# round-3: one-byte stamps in the packed chunk scan -- parity, C3 A/B vs the
# former 20.8 kB per unit (frontier_wg_lds pad)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_bench_size.py -k "fabric or route_stream or packed or c3 or wan" > gpurun_out/u8_tests.log 2>&1; rc=$?; tail -3 gpurun_out/u8_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=10 bash tools/gpu_c3_ab.sh frontier_wg_lds=0 frontier_wg_lds=20800 frontier_wg_lds=0 frontier_wg_lds=20800

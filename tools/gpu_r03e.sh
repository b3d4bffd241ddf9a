#!/bin/bash
# round-3: one-phase packed chunk scan -- parity (parity file + variants), C3 A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_variants.py > gpurun_out/packed_tests.log 2>&1; rc=$?; tail -4 gpurun_out/packed_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=10 bash tools/gpu_c3_ab.sh spf_packed_scan=1 spf_packed_scan=0 spf_packed_scan=1 spf_packed_scan=0

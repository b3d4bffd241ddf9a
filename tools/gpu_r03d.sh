#!/bin/bash
# round-3: batched chunk-record scan in the frontier SPF -- parity, C3 A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "route_stream or fabric or multi_source" > gpurun_out/scan_tests.log 2>&1; rc=$?; tail -4 gpurun_out/scan_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=10 bash tools/gpu_c3_ab.sh spf_scan_batch=1 spf_scan_batch=0 spf_scan_batch=1 spf_scan_batch=0

#!/bin/bash
# round-3: pipelined split route stream (route_stream 3) -- parity, then C3 A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "route_stream" > gpurun_out/rs_tests.log 2>&1; rc=$?; tail -8 gpurun_out/rs_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=10 bash tools/gpu_c3_ab.sh route_stream=2 route_stream=3,route_stream_chunks=2 route_stream=3,route_stream_chunks=4 route_stream=3,route_stream_chunks=8 route_stream=3,route_stream_chunks=16 route_stream=1 route_stream=2

#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -25 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
PPN=1 bash tools/gpu_c3.sh && OGS_UNIT_WIDTH=0 PPN=1 bash tools/gpu_c3.sh && PPN=100 PROF=1 bash tools/gpu_c3.sh

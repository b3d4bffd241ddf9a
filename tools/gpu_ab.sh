#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
OGS_LIB_B=$PWD/openr_amd/lib/libopenr_gpu_base.so VARIANTS=${VARIANTS:-1p#b,1p,1pi,1} timeout -k 10 300 python tools/ab_unit_width.py > gpurun_out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; cat gpurun_out/ab.log | grep -v amdgpu.ids
exit $rc

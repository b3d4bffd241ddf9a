#!/bin/bash
# C2 wave kernel A/B: wave parity tests, then the shipped lib against
# libopenr_gpu_base.so (same process, interleaved), then phase stamps of
# both diagnostic builds. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/openr_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_wave.log 2>&1 || { tail -30 gpurun_out/pytest_wave.log; exit 1; }
tail -2 gpurun_out/pytest_wave.log
OGS_LIB_B=$L/libopenr_gpu_base.so VARIANTS=${VARIANTS:-1pi#b,1pi} timeout -k 10 300 \
  python tools/ab_unit_width.py > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
grep variant= gpurun_out/ab.log
for v in base new; do
  lib=$L/libopenr_gpu_stamps.so; [ $v = base ] && lib=$L/libopenr_gpu_stamps_base.so
  OGS_LIB=$lib WAVE_OPTS=2 VARIANTS=1pi timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps_$v.log 2>&1 || { tail -20 gpurun_out/stamps_$v.log; exit 1; }
  echo "== stamps $v"; grep -v amdgpu.ids gpurun_out/stamps_$v.log
done

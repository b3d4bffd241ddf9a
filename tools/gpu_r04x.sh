#!/bin/bash
# Batched image staging: parity, stamps, timing.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "route_stream" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04x_par.log 2>&1 || { tail -40 gpurun_out/r04x_par.log; exit 1; }
tail -1 gpurun_out/r04x_par.log
OGS_LIB=openr_amd/lib/libopenr_gpu_stamps.so timeout -k 10 200 python -u tools/c3_stamps.py --lds --as-rank 0/8 --opt route_stream=4 > gpurun_out/st.log 2>&1 || { tail -30 gpurun_out/st.log; exit 1; }
grep -v amdgpu.ids gpurun_out/st.log
for r in 0/8 0/1; do
  echo "=== $r"
  timeout -k 10 300 python -u tools/c3_opt_ab.py --pairs 3 --as-rank $r route_stream=5 lds_tail=0 > gpurun_out/r04x_ab.log 2>&1 || { tail -30 gpurun_out/r04x_ab.log; exit 1; }
  grep '^{' gpurun_out/r04x_ab.log | cut -c1-150
done

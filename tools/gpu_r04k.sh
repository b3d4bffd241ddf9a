#!/bin/bash
# Round 4: LDS SPF phase stamps (diagnostic build).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=openr_amd/lib/libopenr_gpu_stamps.so
for r in 0/8 0/1; do
  echo "=== lds stamps $r"
  OGS_LIB=$S timeout -k 10 200 python -u tools/c3_stamps.py --lds --as-rank $r --opt route_stream=4 > gpurun_out/st.log 2>&1 || { tail -30 gpurun_out/st.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/st.log
done

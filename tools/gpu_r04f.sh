#!/bin/bash
# Round 4: phase stamps (diagnostic build) of the C3 launches per geometry.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=openr_amd/lib/libopenr_gpu_stamps.so
st() {
  echo "=== stamps $*"
  OGS_LIB=$S timeout -k 10 200 python -u tools/c3_stamps.py "$@" > gpurun_out/st.log 2>&1 || { tail -30 gpurun_out/st.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/st.log
}
st --as-rank 0/8 --opt frontier_block=512 --opt frontier_parts=2 --opt frontier_parts_wide=4
st --as-rank 0/8 --opt frontier_block=512 --opt frontier_parts=1 --opt frontier_parts_wide=1
st --as-rank 0/8 --opt frontier_block=256 --opt frontier_parts=1 --opt frontier_parts_wide=1
st --as-rank 0/8 --opt frontier_block=1024 --opt frontier_parts=1 --opt frontier_parts_wide=1
echo "=== projection (auto geometry)"
timeout -k 10 400 python -u bench.py --config c3 --steps 20 --no-cpu-baseline --no-extras > gpurun_out/r04f_proj.json 2> gpurun_out/r04f_proj.log || { tail -30 gpurun_out/r04f_proj.log; exit 1; }
grep "c3 " gpurun_out/r04f_proj.log

#!/bin/bash
# Round 4: phase stamps of the C3 fused launches at shard sizes (diagnostic
# build) + kernel trace of the split SPF / stream form on the N=8 shard.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=openr_amd/lib/libopenr_gpu_stamps.so
for cfg in "0/8 frontier_block=256" "0/8 frontier_block=1024" "0/4 frontier_block=512" "0/1 frontier_block=256"; do
  set -- $cfg
  echo "=== stamps shard $1 $2"
  OGS_LIB=$S timeout -k 10 200 python -u tools/c3_stamps.py --as-rank $1 --opt $2 > gpurun_out/st.log 2>&1 || { tail -30 gpurun_out/st.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/st.log
done
cd /tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r8 -o r8 -- python3 tools/c3_opt_ab.py --pairs 1 --steps 5 --as-rank 0/8 frontier_block=256 frontier_block=1024 route_stream=1 > gpurun_out/prof_r8.log 2>&1 || { tail -20 gpurun_out/prof_r8.log; exit 1; }
grep '^{' gpurun_out/prof_r8.log
grep -v "at::native" gpurun_out/prof_r8/r8_kernel_stats.csv | cut -c1-250

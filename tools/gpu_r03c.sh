#!/bin/bash
# round-3: C3 SPF-form A/B (spf_queue) and a kernel trace of the pipelined split
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=10 bash tools/gpu_c3_ab.sh route_stream=2 spf_queue=1 spf_queue=2 spf_ninfo=0 route_stream=2 || exit $?
cd /tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3p -o c3p -- python3 bench.py --config c3 --no-cpu-baseline --no-extras --steps 3 --warmup 1 --opt route_stream=3 --opt route_stream_chunks=2 > gpurun_out/rocprof_c3p.log 2>&1 || exit $?
grep -v "at::native" gpurun_out/prof_c3p/c3p_kernel_stats.csv | cut -c1-90,150-

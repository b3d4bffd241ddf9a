#!/bin/bash
# Config C5 on the GPU box: bench line + rocprofv3 kernel stats.
# usage (via gpurun): bash tools/gpu_c5.sh [extra bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 "$@" > gpurun_out/c5.log 2>&1 || { tail -5 gpurun_out/c5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o c5 -- python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/c5prof.log 2>&1 || { tail -5 gpurun_out/c5prof.log; exit 1; }
tail -1 gpurun_out/c5.log

#!/bin/bash
# C3 fabric all-sources bench (+ kernel-trace profile). UW selects the kernel
# (unit_width option via OGS_UNIT_WIDTH), MSG the multi-source grouping.
mkdir -p gpurun_out; export TMPDIR=/tmp
PPN=${PPN:-100}
timeout -k 10 600 python bench.py --config c3 --prefixes-per-node $PPN --steps ${STEPS:-3} --warmup 1 > gpurun_out/bench_c3.log 2>&1 || { tail -20 gpurun_out/bench_c3.log; exit 1; }
grep '^{' gpurun_out/bench_c3.log | cut -c1-900
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --config c3 --prefixes-per-node $PPN --steps 2 --warmup 1 > gpurun_out/rocprof_c3.log 2>&1 || exit $?
  grep -v "at::native" gpurun_out/prof_c3/c3_kernel_stats.csv
fi

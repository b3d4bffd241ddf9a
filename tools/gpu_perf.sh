#!/bin/bash
# stamps (diagnostic lib) + bench + kernel-trace profile of the shipped lib
mkdir -p gpurun_out; export TMPDIR=/tmp
OGS_LIB=$PWD/openr_amd/lib/libopenr_gpu_stamps.so VARIANTS=1p,1pi timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps.log
timeout -k 10 600 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1 || exit $?
cat gpurun_out/prof/bench_kernel_stats.csv

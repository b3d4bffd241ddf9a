#!/bin/bash
# C3 A/B: chunk records of 8 edges (default build) vs 16 (OGS_LIB=
# openr_amd/lib/libopenr_gpu_chunk16.so, spf_frontier.hip -DOGS_CHUNK_EDGES=16)
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 8 16 8 16; do  # 16 = the OGS_LIB variant build (any -DOGS_CHUNK_EDGES)
  if [ $v = 16 ]; then L=openr_amd/lib/libopenr_gpu_chunk16.so; else L=openr_amd/lib/libopenr_gpu.so; fi
  OGS_LIB=$L timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-extras --steps 10 --warmup 2 > gpurun_out/bench_chunk_ab.log 2>&1 || { tail -5 gpurun_out/bench_chunk_ab.log; exit 1; }
  grep '^{' gpurun_out/bench_chunk_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk=$v', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['golden'])"
done

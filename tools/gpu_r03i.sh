#!/bin/bash
# round-3: KSP2 stack / queue overlay -- parity, C5 A/B over ksp_stage
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ksp_domains.py tests/test_gpu_parity.py tests/test_gpu_bench_size.py tests/test_gpu_fuzz.py -k "ksp or c5 or KSP" > gpurun_out/ksp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ksp_tests.log; [ $rc -eq 0 ] || exit $rc
for v in -1 0 -1 0; do
  timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-extras --opt ksp_stage=$v > gpurun_out/bench_c5_ab.log 2>&1 || { tail -5 gpurun_out/bench_c5_ab.log; exit 1; }
  grep '^{' gpurun_out/bench_c5_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ksp_stage=$v', d['ms_per_step'], d['ksp2_kernels_ms'], d['job_kernel_ms'], d['golden'])"
done

#!/bin/bash
# spf_ninfo: parity under both settings, then C4 / C5 A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/ninfo_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ninfo_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  timeout -k 10 200 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --opt spf_ninfo=$v > gpurun_out/ninfo_c4.log 2>&1 || exit $?
  echo "c4 spf_ninfo=$v: $(grep '^{' gpurun_out/ninfo_c4.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['kernel_ms'], l['route_digest'])")"
done
for v in 1 0; do
  timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --opt spf_ninfo=$v > gpurun_out/ninfo_c5.log 2>&1 || exit $?
  echo "c5 spf_ninfo=$v: $(grep '^{' gpurun_out/ninfo_c5.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['route_kernels_ms'], l['path_digest'])")"
done

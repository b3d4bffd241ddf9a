#!/bin/bash
# folded push stamps (QMODE 3, default) vs packed form 2 (spf_queue=3): parity, C4/C5 A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/fold_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fold_tests.log; [ $rc -eq 0 ] || exit $rc
for v in -1 3 -1 3; do
  timeout -k 10 200 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --opt spf_queue=$v > gpurun_out/fold_c4.log 2>&1 || exit $?
  echo "c4 spf_queue=$v: $(grep '^{' gpurun_out/fold_c4.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['kernel_ms'], l['route_digest'])")"
done
for v in -1 3; do
  timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --opt spf_queue=$v > gpurun_out/fold_c5.log 2>&1 || exit $?
  echo "c5 spf_queue=$v: $(grep '^{' gpurun_out/fold_c5.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['route_kernels_ms'], l['path_digest'])")"
done

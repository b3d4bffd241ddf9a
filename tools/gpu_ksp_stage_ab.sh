#!/bin/bash
# A/B of the KSP2 staging level on the C5 job (same results, different LDS/unit)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for st in 0 1 2; do
  timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --opt ksp_stage=$st > gpurun_out/ksp_st$st.log 2>&1 || exit $?
  echo "ksp_stage=$st"; grep '^{' gpurun_out/ksp_st$st.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['ksp2_kernels_ms'], l['path_digest'])"
done

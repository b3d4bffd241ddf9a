#!/bin/bash
# KSP2 batch variants: parity tests, then the C5 line per option set.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "ksp or c5 or kat" > gpurun_out/k_pytest.log 2>&1 || { tail -30 gpurun_out/k_pytest.log; exit 1; }
tail -2 gpurun_out/k_pytest.log
i=0
for opts in "--opt ksp_stage=-1" "--opt ksp_stage=0" "--opt ksp_stage=2" "--opt ksp_queue=0"; do
  i=$((i+1))
  timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline \
    $opts > gpurun_out/k_c5_$i.log 2>&1 || { tail -5 gpurun_out/k_c5_$i.log; exit 1; }
  echo "$opts: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/k_c5_$i.log | head -1) \
$(grep -o '"ksp2_kernels_ms": [0-9.]*' gpurun_out/k_c5_$i.log | head -1) \
$(grep -o '"path_digest": "[0-9a-f]*"' gpurun_out/k_c5_$i.log | head -1)"
done

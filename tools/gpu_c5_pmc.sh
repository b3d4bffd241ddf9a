#!/bin/bash
# C5: KSP parity tests, bench line, kernel stats, PMC passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "ksp or c5 or kat or policy" > gpurun_out/k_pytest.log 2>&1 || { tail -30 gpurun_out/k_pytest.log; exit 1; }
tail -1 gpurun_out/k_pytest.log
bash tools/gpu_c5.sh || exit $?
bash tools/gpu_pmc.sh c5 --config c5 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/pmc_c5.txt 2>&1 || { tail -5 gpurun_out/pmc_c5.txt; exit 1; }

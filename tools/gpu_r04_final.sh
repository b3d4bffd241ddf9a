#!/bin/bash
# Round-4 evidence at HEAD in one call: full GPU suite, smoke, default bench,
# kernel trace of the bench, PMC passes (C3, C2, C4, C5, G1). Stops at the
# first failure. OGS_COMMIT=<sha> names the commit in the PMC summaries.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 420 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 420 python bench.py
cd /tmp && cd "$GRAFT_REPO_ROOT"
step rocprof 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --no-cpu-baseline --no-extras
bash tools/gpu_round_pmc.sh > gpurun_out/pmc_round.log 2>&1 || { tail -5 gpurun_out/pmc_round.log; exit 1; }
echo "=== pmc done"

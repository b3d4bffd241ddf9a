#!/bin/bash
# The round-end sequence on one GPU box: parity tests, smoke, default bench,
# kernel-trace profile of the default bench. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
nproc > gpurun_out/host.txt; python3 -c "import os;print(len(os.sched_getaffinity(0)))" >> gpurun_out/host.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/host.txt 2>/dev/null; lscpu | grep "Model name" >> gpurun_out/host.txt
if [ -z "$NO_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 900 python bench.py
if [ -n "$PROFILE" ]; then
  cd /tmp && cd "$GRAFT_REPO_ROOT"
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --no-cpu-baseline --no-extras
  grep -v "at::native" gpurun_out/prof/bench_kernel_stats.csv | cut -c1-200
fi

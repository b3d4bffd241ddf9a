#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.
# Stops at the first step that ends in anything but success / test failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
nproc > gpurun_out/host.txt; lscpu | grep "Model name" >> gpurun_out/host.txt
step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x ${PYTEST_ARGS}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 50 --warmup 5
if [ -n "$PROFILE" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
fi
exit 0

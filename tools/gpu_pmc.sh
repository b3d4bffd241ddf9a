#!/bin/bash
# HBM traffic of the bench's dominant kernel from PMC counters, per
# MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE in separate
# passes (TCC slots), each pass its own short run; the summary is written by
# tools/pmc_summary.py. Usage: tools/gpu_pmc.sh <tag> <bench args...>
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${tag}_$c -o pmc -- python3 bench.py "$@" > gpurun_out/pmc_${tag}_$c.log 2>&1 || { echo "pmc pass $c failed"; tail -5 gpurun_out/pmc_${tag}_$c.log; exit 1; }
done
python3 tools/pmc_summary.py $tag "$@"

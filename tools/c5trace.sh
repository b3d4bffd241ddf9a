#!/bin/bash
# C5 kernel + copy trace per process-group variant: which
# hardware queue each stream's dispatches land on. Args: bench flag sets,
# e.g. "--dist auto" "--dist none" "--dist auto --early-streams 0".
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for v in "$@"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/c5tr_$i -o c5 -- python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline $v > gpurun_out/c5tr_$i.log 2>&1 || exit $?
  echo "[$v] $(grep '^{' gpurun_out/c5tr_$i.log | cut -c1-160)"
done

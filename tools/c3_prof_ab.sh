#!/bin/bash
# Does the kernel-trace profiler change the C3 headline? The same bench runs
# with and without rocprofv3 --kernel-trace, interleaved (round 6: the
# profiled default line measured 1.00 ms/build against 1.09 unprofiled).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
A="--config c3 --no-cpu-baseline --no-shard-projection --steps 20 --warmup 3"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $A > gpurun_out/c3pa_plain_$rep.log 2>&1 || exit $?
  echo "plain $rep: $(grep -o 'c3 timed: [0-9.]* ms' gpurun_out/c3pa_plain_$rep.log)"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3pa_kt_$rep -o kt -- python3 bench.py $A > gpurun_out/c3pa_kt_$rep.log 2>&1 || exit $?
  echo "ktrace $rep: $(grep -o 'c3 timed: [0-9.]* ms' gpurun_out/c3pa_kt_$rep.log)"
  timeout -k 10 300 python3 bench.py $A --dist none > gpurun_out/c3pa_none_$rep.log 2>&1 || exit $?
  echo "plain --dist none $rep: $(grep -o 'c3 timed: [0-9.]* ms' gpurun_out/c3pa_none_$rep.log)"
done

#!/bin/bash
# C5 job on one vs two HIP streams (RouteDb+policy || KSP2); same digest
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for n in 1 2 1 2; do
  timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --c5-streams $n > gpurun_out/c5s.log 2>&1 || exit $?
  echo "c5 streams=$n: $(grep '^{' gpurun_out/c5s.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['ms_per_step'], l['path_digest'])")"
done

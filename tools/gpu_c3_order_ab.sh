#!/bin/bash
# A/B of the C3 width-group dispatch order (and single stream), same results
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "--c3-order narrow-first" "--c3-order wide-first" "--c3-order wide-first --c3-streams 1" "--c3-order narrow-first" "--c3-order wide-first"; do
  timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 $cfg > gpurun_out/c3ab.log 2>&1 || exit $?
  echo "$cfg: $(grep '^{' gpurun_out/c3ab.log | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['ms_per_step'], l['route_digest'])")"
done

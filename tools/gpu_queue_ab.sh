#!/bin/bash
# Queue-form frontier SPF: parity tests, then C4 / C5 lines with the queue
# form (default) and with the chunk scan (spf_queue=0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "variant or wan or multi_area or c5 or fabric or policy" > gpurun_out/q_pytest.log 2>&1 \
  || { tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -2 gpurun_out/q_pytest.log
for opt in "spf_queue=-1" "spf_queue=2"; do
  for cfg in c4 c5; do
    timeout -k 10 300 python3 -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline \
      --opt $opt > gpurun_out/q_${cfg}_${opt}.log 2>&1 || { tail -5 gpurun_out/q_${cfg}_${opt}.log; exit 1; }
    echo "$cfg $opt $(grep -o '"value": [0-9.]*' gpurun_out/q_${cfg}_${opt}.log | head -1) \
$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q_${cfg}_${opt}.log | head -1) \
$(grep -o '"route_kernels_ms": [0-9.]*' gpurun_out/q_${cfg}_${opt}.log | head -1)"
  done
done

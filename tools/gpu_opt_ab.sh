#!/bin/bash
# One engine option A/B'd on bench lines, values interleaved, then GPU tests.
#   OPT=route_store_nt VALS="1 0 1 0" CONFIGS="c2 c3" STEPS=10 K="store" \
#     bash tools/gpu_opt_ab.sh
# (NOTEST=1 skips the tests)
mkdir -p gpurun_out; export TMPDIR=/tmp
OPT=${OPT:-route_store_nt}
for cfg in ${CONFIGS:-c3}; do
  for val in ${VALS:-1 0 1 0}; do
    echo "=== $cfg $OPT=$val"
    timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extras --opt $OPT=$val > gpurun_out/opt_ab.log 2>&1 || { tail -20 gpurun_out/opt_ab.log; exit 1; }
    grep '^{' gpurun_out/opt_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('kernel_ms'), d['roofline']['frac'])"
  done
done
[ -n "$NOTEST" ] && exit 0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py ${TEST_FILES} -k "${K:-store_flavours or wave or route_stream}" > gpurun_out/opt_tests.log 2>&1 || { tail -30 gpurun_out/opt_tests.log; exit 1; }
tail -2 gpurun_out/opt_tests.log

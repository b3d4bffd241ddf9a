#!/bin/bash
# C4 A/B: bench c4 with openr_amd/lib/libopenr_gpu_base.so (tools/build_ab_base.sh REV spf_frontier)
# against the working-tree build, interleaved, then the variant parity tests.
mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
for i in 1 2; do
 for L in base new; do
  if [ $L = base ]; then export OGS_LIB=$PWD/openr_amd/lib/libopenr_gpu_base.so; else unset OGS_LIB; fi
  timeout -k 10 180 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/c4_$L$i.json 2>gpurun_out/c4_$L$i.err || exit $?
  echo "$L$i $(tail -1 gpurun_out/c4_$L$i.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["ms_per_step"],d.get("golden"),d.get("roofline",{}).get("frac"))')"
 done
done
unset OGS_LIB
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_variants.py tests/test_gpu_bench_size.py -p no:cacheprovider > gpurun_out/c4_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/c4_pytest.log; exit $rc

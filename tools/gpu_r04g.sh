#!/bin/bash
# Round 4: parity of the SPF memo / incremental batch / geometry changes,
# phase stamps at N = 8, and the C3 line with its shard projection.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_counters.py tests/test_gpu_incremental_routes.py tests/test_gpu_bench_size.py -k "not c4 and not c5" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1 || { tail -40 gpurun_out/r04g_tests.log; exit 1; }
tail -3 gpurun_out/r04g_tests.log
S=openr_amd/lib/libopenr_gpu_stamps.so
for o in "" "--opt frontier_block=512 --opt frontier_parts=1 --opt frontier_parts_wide=1"; do
  echo "=== stamps 0/8 $o"
  OGS_LIB=$S timeout -k 10 200 python -u tools/c3_stamps.py --as-rank 0/8 $o > gpurun_out/st.log 2>&1 || { tail -30 gpurun_out/st.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/st.log
done
timeout -k 10 600 python -u bench.py --config c3 --steps 20 > gpurun_out/r04g_c3.json 2> gpurun_out/r04g_c3.log || { tail -30 gpurun_out/r04g_c3.log; exit 1; }
grep "c3 " gpurun_out/r04g_c3.log
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r04g_c3.json') if l.startswith('{')][0])
print(d['ms_per_step'], d['roofline']['frac'], d['golden'])
for n,v in d['shard_projection'].items(): print(n, v['ms'], v['frac'], v['min_frac'])
print(d.get('incremental_routes'))"

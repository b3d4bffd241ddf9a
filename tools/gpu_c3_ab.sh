#!/bin/bash
# C3 A/B over engine options: each argument is one bench variant's --opt list
# (comma separated), e.g.  route_stream=1  route_stream=2 ; then a kernel
# trace of the default configuration.
mkdir -p gpurun_out; export TMPDIR=/tmp
PPN=${PPN:-100}
for v in "$@"; do
  opts=""; for o in ${v//,/ }; do case $o in --*) opts="$opts ${o/=/ }";; *) opts="$opts --opt $o";; esac; done
  echo "=== $v"
  timeout -k 10 300 python bench.py --config c3 --prefixes-per-node $PPN --steps ${STEPS:-5} --warmup 1 $opts > gpurun_out/bench_c3_ab.log 2>&1 || { tail -20 gpurun_out/bench_c3_ab.log; exit 1; }
  grep '^{' gpurun_out/bench_c3_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --config c3 --prefixes-per-node $PPN --steps 3 --warmup 1 > gpurun_out/rocprof_c3.log 2>&1 || exit $?
  grep -v "at::native" gpurun_out/prof_c3/c3_kernel_stats.csv | cut -c1-60,150-
fi

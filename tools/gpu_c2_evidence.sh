#!/bin/bash
# C2 evidence at the current tree: SQ wave-cycle pass and a kernel trace of
# a C2-only bench (so spf_route_wave_kernel's average is C2 launches only).
mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
F="--config c2 --no-cpu-baseline --no-extras"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sq_c2 -o sq -- python3 bench.py $F --steps 10 --warmup 2 > gpurun_out/sq_c2.log 2>&1 || { tail -5 gpurun_out/sq_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c2 -o c2 -- python3 bench.py $F --steps 50 --warmup 5 > gpurun_out/kt_c2.log 2>&1 || { tail -5 gpurun_out/kt_c2.log; exit 1; }
tail -1 gpurun_out/kt_c2.log | cut -c1-600
grep -v "at::native" gpurun_out/kt_c2/c2_kernel_stats.csv | cut -c1-200
echo done

#!/bin/bash
# C3 (headline) evidence at the current tree: SQ wave-cycle pass and a
# kernel trace of a C3-only bench (fused spf_frontier_kernel + route stream).
mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
F="--config c3 --no-cpu-baseline --no-extras"
timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sq_c3 -o sq -- python3 bench.py $F --steps 3 --warmup 1 > gpurun_out/sq_c3.log 2>&1 || { tail -5 gpurun_out/sq_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c3 -o c3 -- python3 bench.py $F --steps 20 --warmup 3 > gpurun_out/kt_c3.log 2>&1 || { tail -5 gpurun_out/kt_c3.log; exit 1; }
tail -1 gpurun_out/kt_c3.log | cut -c1-400
grep -v "at::native" gpurun_out/kt_c3/c3_kernel_stats.csv | cut -c1-200
echo done

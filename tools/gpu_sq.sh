#!/bin/bash
# SQ counter pass (wave-cycle breakdown, LDS conflicts) for C2 and C4
mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sq_c2 -o sq -- python3 bench.py --config c2 --no-cpu-baseline --no-extras --steps 10 --warmup 2 > gpurun_out/sq_c2.log 2>&1 || { tail -5 gpurun_out/sq_c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sq_c4 -o sq -- python3 bench.py --config c4 --no-cpu-baseline --no-extras --steps 3 --warmup 1 > gpurun_out/sq_c4.log 2>&1 || { tail -5 gpurun_out/sq_c4.log; exit 1; }
echo done

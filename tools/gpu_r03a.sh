#!/bin/bash
# round-3 checks: wave pair form (tests, A/B, C2 line), G1 line, C3
# occupancy A/B (frontier_wg_lds)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_pair.sh || exit $?
STEPS=10 bash tools/gpu_c3_ab.sh frontier_wg_lds=0 frontier_wg_lds=32768 frontier_wg_lds=40960 frontier_wg_lds=54000 frontier_wg_lds=0

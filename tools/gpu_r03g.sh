#!/bin/bash
# round-3 evidence: G1 PMC (batch launches only), C2-alone kernel trace, SQ passes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OGS_COMMIT=$1 bash tools/gpu_pmc.sh g1 --config g1 --no-cpu-baseline --no-extras --steps 1 --warmup 1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c2 -o c2 -- python3 bench.py --config c2 --no-cpu-baseline --no-extras > gpurun_out/kt_c2.log 2>&1 || exit $?
bash tools/gpu_sq.sh || exit $?
python3 tools/sq_summary.py gpurun_out/sq_c2/sq_counter_collection.csv spf_route_wave_kernel gpurun_out/sq_c2.json $1
python3 tools/sq_summary.py gpurun_out/sq_c4/sq_counter_collection.csv spf_variant_repair_kernel gpurun_out/sq_c4.json $1
grep -v "at::native" gpurun_out/kt_c2/c2_kernel_stats.csv | cut -c1-120

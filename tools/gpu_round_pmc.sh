#!/bin/bash
# Round-end evidence: tests + smoke + default bench + kernel-trace profile
# (tools/gpu_round.sh with PROFILE=1), then PMC traffic passes for the C2, C4
# and C5 kernels (tools/gpu_pmc.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PROFILE=1 bash tools/gpu_round.sh || exit $?
bash tools/gpu_pmc.sh c2 --no-c3 --no-c4 --no-c5 --no-cpu-baseline --steps 20 --warmup 3 || exit $?
bash tools/gpu_pmc.sh c4 --config c4 --no-cpu-baseline --steps 3 --warmup 1 || exit $?
bash tools/gpu_pmc.sh c5 --config c5 --no-cpu-baseline --steps 5 --warmup 1 || exit $?

#!/bin/bash
# Round-end PMC evidence: HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one
# run each, tools/gpu_pmc.sh) for the C2, C3, C4 and C5 dominant kernels.
# Run tools/gpu_round.sh (PROFILE=1) first for tests / smoke / bench / trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
F="--no-cpu-baseline --no-c1 --no-g1 --no-extras"
bash tools/gpu_pmc.sh c2 --no-c3 --no-c4 --no-c5 $F --steps 20 --warmup 3 || exit $?
bash tools/gpu_pmc.sh c3 --config c3 $F --steps 2 --warmup 1 || exit $?
bash tools/gpu_pmc.sh c4 --config c4 $F --steps 3 --warmup 1 || exit $?
bash tools/gpu_pmc.sh c5 --config c5 $F --steps 5 --warmup 1 || exit $?
bash tools/gpu_pmc.sh g1 --no-c3 --no-c4 --no-c5 --no-cpu-baseline --no-c1 --steps 1 --warmup 1 || exit $?

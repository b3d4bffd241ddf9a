#!/bin/bash
# Round-end PMC evidence: HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one
# run each, tools/gpu_pmc.sh) for the dominant kernels of C3 (headline), C2,
# C4, C5 and G1. Call as `OGS_COMMIT=<sha> bash tools/gpu_round_pmc.sh` so
# each summary records the commit it measured.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
F="--no-cpu-baseline --no-extras"
bash tools/gpu_pmc.sh c3 --config c3 $F --no-shard-projection --steps 2 --warmup 1 || exit $?
bash tools/gpu_pmc.sh c2 --config c2 $F --steps 20 --warmup 3 || exit $?
bash tools/gpu_pmc.sh c4 --config c4 $F --steps 3 --warmup 1 || exit $?
bash tools/gpu_pmc.sh c5 --config c5 $F --steps 5 --warmup 1 || exit $?
bash tools/gpu_pmc.sh g1 --config g1 $F --steps 1 --warmup 1 || exit $?

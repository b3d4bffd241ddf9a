#!/bin/bash
# C3 PMC passes (HBM traffic) at HEAD for the one-launch form.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_pmc.sh c3 --config c3 --no-cpu-baseline --no-extras --no-shard-projection --steps 2 --warmup 1 || exit $?
cat gpurun_out/pmc_c3.json | head -40

#!/bin/bash
# Round evidence: tests + smoke + default bench + kernel trace + PMC passes,
# then the N=2 shared-device rehearsal of the multi-rank path.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round_pmc.sh || exit $?
bash tools/gpu_rehearse_n2.sh

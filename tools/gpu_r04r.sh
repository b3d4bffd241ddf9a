#!/bin/bash
# Full GPU suite at HEAD (route_stream 5 default), then smoke.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r04r_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r04r_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04r_smoke.log 2>&1 || { tail -20 gpurun_out/r04r_smoke.log; exit 1; }
tail -3 gpurun_out/r04r_smoke.log

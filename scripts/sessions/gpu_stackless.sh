#!/bin/bash
# stackless brute-force replay: the GPU suite, then an in-process A/B against the stack walk
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02q}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/env_ab.py --spp 64 --reps 5 'PT_BF_STACKLESS=1' 'PT_BF_STACKLESS=0' 'PT_BF_STACKLESS=1' > gpurun_out/${TAG}_ab.log 2>&1
rc=$?; tail -6 gpurun_out/${TAG}_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/env_ab.py --scene CornellBox-Mirror --depth 16 --spp 64 --reps 5 'PT_BF_STACKLESS=0' 'PT_BF_STACKLESS=1' > gpurun_out/${TAG}_ab_mirror.log 2>&1
rc=$?; tail -6 gpurun_out/${TAG}_ab_mirror.log; exit $rc

#!/bin/bash
# traversal-kernel change: GPU suite, then the traversal scenes in-process
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02dyn}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/env_ab.py --scene CornellBox-Glossy --depth 16 --spp 32 --reps 2 'PT_PARTS=2' 'PT_PARTS=1' 'PT_PARTS=4' > gpurun_out/${TAG}_ab_glossy.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_ab_glossy.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --depth 16 --spp 8 --reps 2 'PT_PARTS=2' 'PT_PARTS=1' > gpurun_out/${TAG}_ab_boat.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_ab_boat.log; exit $rc

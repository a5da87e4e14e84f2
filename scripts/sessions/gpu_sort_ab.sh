#!/bin/bash
# octant grouping of survivors (PT_SORT): parity subset, then A/B on the traversal scenes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02w}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "sort" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/env_ab.py --scene CornellBox-Glossy --depth 16 --spp 32 --reps 2 'PT_SORT=0' 'PT_SORT=8' 'PT_SORT=64' 'PT_SORT=0' 'PT_SORT=64' > gpurun_out/${TAG}_ab_glossy.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_ab_glossy.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --depth 16 --spp 8 --reps 2 'PT_SORT=0' 'PT_SORT=8' 'PT_SORT=64' > gpurun_out/${TAG}_ab_boat.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_ab_boat.log; exit $rc

#!/bin/bash
# cooperative big-leaf turns (PT_BIG_LEAF=n): parity subset, then A/B on the boat
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02big}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "big or tie" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --depth 16 --spp 8 --reps 2 'PT_BIG_LEAF=0' 'PT_BIG_LEAF=256' 'PT_BIG_LEAF=1024' 'PT_BIG_LEAF=64' 'PT_BIG_LEAF=0' > gpurun_out/${TAG}_ab_boat.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_ab_boat.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/env_ab.py --scene CornellBox-Glossy --depth 16 --spp 16 --reps 2 'PT_BIG_LEAF=0' 'PT_BIG_LEAF=32' > gpurun_out/${TAG}_ab_glossy.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_ab_glossy.log; exit $rc

#!/bin/bash
# camera paths in 8x8 tiles (option tiles) vs row order: parity variants, then in-process A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -k "tiles" -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/tiles_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/tiles_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_tiles.log
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox-Glossy --spp 32 --depth 16 --reps 3 tiles=0 tiles=1 >> gpurun_out/ab_tiles.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox --spp 64 --depth 8 --reps 3 tiles=0 tiles=1 >> gpurun_out/ab_tiles.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --spp 8 --depth 16 --reps 2 tiles=0 tiles=1 >> gpurun_out/ab_tiles.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --synthetic 1000 --spp 16 --depth 8 --reps 3 tiles=0 tiles=1 >> gpurun_out/ab_tiles.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_tiles.log

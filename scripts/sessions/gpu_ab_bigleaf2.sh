#!/bin/bash
# cooperative big-leaf threshold (option big_leaf) on the traversal scenes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
: > gpurun_out/ab_bigleaf2.log
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox-Glossy --spp 32 --depth 16 --reps 3 big_leaf=128 big_leaf=48 big_leaf=32 big_leaf=24 big_leaf=16 >> gpurun_out/ab_bigleaf2.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox-Sphere --spp 32 --depth 16 --reps 3 big_leaf=128 big_leaf=32 big_leaf=16 >> gpurun_out/ab_bigleaf2.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 8 --depth 16 --reps 2 big_leaf=128 big_leaf=64 big_leaf=32 >> gpurun_out/ab_bigleaf2.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_bigleaf2.log

#!/bin/bash
# leaf chunks: stress test (chunk_leaf == sequential loop), parity (leaf variants, boat frames, boat band), A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T="--timeout 250 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_leafbvh.py -v -s $T > gpurun_out/leaf_stress.log 2>&1
rc=$?; tail -3 gpurun_out/leaf_stress.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -k "leaf or MedievalBoat" $T > gpurun_out/leaf_parity.log 2>&1
rc=$?; tail -3 gpurun_out/leaf_parity.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_leaf.log
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 8 --depth 16 --reps 2 --scene-opt leaf_bvh=128 leaf_walk=0 leaf_walk=1 >> gpurun_out/ab_leaf.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 8 --depth 16 --reps 2 --scene-opt leaf_bvh=64 leaf_walk=0 leaf_walk=1 >> gpurun_out/ab_leaf.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --spp 16 --depth 16 --reps 3 --scene-opt leaf_bvh=128 leaf_walk=0 leaf_walk=1 >> gpurun_out/ab_leaf.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_leaf.log

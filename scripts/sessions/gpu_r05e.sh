#!/bin/bash
# Round 5: big-leaf keys applied inside the leaf turns (no parking turns); the leaf pass as before.
# big-leaf / leaf-BVH variants incl. the new leafpass ones, the boat bands with leaf_pre on/off,
# the fast trees), then the boat A/B in process (leaf_pre 1 vs 0) and its config line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05e_pytest_parity.log 2>&1
rc=$?; tail -3 $P/r05e_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_config_bands.py tests/test_gpu_leafbvh.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "boat or leaf" > $P/r05e_pytest_boat.log 2>&1
rc=$?; tail -3 $P/r05e_pytest_boat.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 960 --spp 8 --depth 16 --reps 3 --profile 'leaf_pre=1' 'leaf_pre=0' 'leaf_cull=1' > $P/r05e_ab_leafpre.log 2>&1
rc=$?; cat $P/r05e_ab_leafpre.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene MedievalBoat --width 1920 --height 1080 --spp 512 --depth 16 > $P/r05e_boat.json 2>&1
rc=$?; echo "boat rc=$rc"; cut -c1-200 $P/r05e_boat.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 600 --timeout-method thread > $P/r05e_pytest_gpu.log 2>&1
rc=$?; tail -3 $P/r05e_pytest_gpu.log; exit $rc

#!/bin/bash
# Round 5: AUTO's choice of the leaf pass by the camera probe (render_impl, probe_pre_leaves): the
# leaf-pass parity variants (forced with leaf_pre=1), the boat and CornellBox2-all-meshes bands, and
# the A/B of the default against leaf_pre=0 / 1 on both scenes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05m_pytest_parity.log 2>&1
rc=$?; tail -2 $P/r05m_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_config_bands.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread -k "boat or cornellbox2" > $P/r05m_pytest_bands.log 2>&1
rc=$?; tail -2 $P/r05m_pytest_bands.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/env_ab.py --scene CornellBox2 --all-meshes --width 1024 --height 1024 --spp 4 --depth 16 --reps 2 '' 'leaf_pre=0' 'leaf_pre=1' > $P/r05m_ab_cb2.log 2>&1
rc=$?; tail -4 $P/r05m_ab_cb2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 960 --spp 8 --depth 16 --reps 2 '' 'leaf_pre=0' 'leaf_pre=1' > $P/r05m_ab_boat.log 2>&1
rc=$?; tail -4 $P/r05m_ab_boat.log; [ $rc -eq 0 ] || exit $rc

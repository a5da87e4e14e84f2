#!/bin/bash
# Round 5: the pass's chunks merged up to 16 by default — leaf-pass parity, boat / CornellBox2 bands
# and fast trees; in process against 24-entry merged chunks (ablib/m16_24).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05al_pytest_parity.log 2>&1
rc=$?; tail -2 $P/r05al_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_config_bands.py tests/test_gpu_fast_trees.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > $P/r05al_pytest_bands.log 2>&1
rc=$?; tail -2 $P/r05al_pytest_bands.log; [ $rc -eq 0 ] || exit $rc
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/m16_24/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 > $P/r05al_ab_merge24.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py ablib/m16_24/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 >> $P/r05al_ab_merge24.log 2>&1
rc=$?; grep '"lib"' $P/r05al_ab_merge24.log; [ $rc -eq 0 ] || exit $rc

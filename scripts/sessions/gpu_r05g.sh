#!/bin/bash
# Round 5: the leaf pass with two entries per step (LDS reads ahead) and the reciprocal-free vote,
# against the previous build (ablib/r05e) in one process, both orders; parity of the leaf variants
# and the boat bands first.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05g_pytest_parity.log 2>&1
rc=$?; tail -2 $P/r05g_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_config_bands.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "boat or cornellbox2" > $P/r05g_pytest_boat.log 2>&1
rc=$?; tail -2 $P/r05g_pytest_boat.log; [ $rc -eq 0 ] || exit $rc
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py ablib/r05e/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 > $P/r05g_ab_leafpass.log 2>&1
rc=$?; cat $P/r05g_ab_leafpass.log | grep lib; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/r05e/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 >> $P/r05g_ab_leafpass.log 2>&1
rc=$?; tail -2 $P/r05g_ab_leafpass.log; exit $rc

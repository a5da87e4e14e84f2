#!/bin/bash
# Round 5: the leaf pass's (ray, chunk) pair walk of chunked leaves (option leaf_pairs): parity of the
# leaf variants and the boat / CornellBox2 bands, then in one process against ablib/r05i (the whole-leaf
# walk at 8 waves) and against itself with leaf_pairs=0.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05j_pytest_parity.log 2>&1
rc=$?; tail -2 $P/r05j_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_config_bands.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "boat or cornellbox2" > $P/r05j_pytest_boat.log 2>&1
rc=$?; tail -2 $P/r05j_pytest_boat.log; [ $rc -eq 0 ] || exit $rc
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py ablib/r05i/libpt_hip.so $L "$L@leaf_pairs=0" --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 > $P/r05j_ab_pairs.log 2>&1
rc=$?; grep lib $P/r05j_ab_pairs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py "$L@leaf_pairs=0" $L ablib/r05i/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 >> $P/r05j_ab_pairs.log 2>&1
rc=$?; tail -3 $P/r05j_ab_pairs.log; exit $rc

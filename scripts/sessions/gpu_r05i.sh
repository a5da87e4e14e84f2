#!/bin/bash
# Round 5: leaf pass at 8 waves (record blocks of 16, the chunk walk removed; ablib/r05i) and with the ray wait hoisted out of the entry loop (the build), against ablib/r05e, one process.
# (ablib/r05e: one entry per step; ablib/r05g: two per step + reciprocal-free vote), one process.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05i_pytest_parity.log 2>&1
rc=$?; tail -2 $P/r05i_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py ablib/r05e/libpt_hip.so ablib/r05i/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 > $P/r05i_ab_leafpass.log 2>&1
rc=$?; grep lib $P/r05i_ab_leafpass.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/r05i/libpt_hip.so ablib/r05e/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 >> $P/r05i_ab_leafpass.log 2>&1
rc=$?; tail -3 $P/r05i_ab_leafpass.log; exit $rc

#!/bin/bash
# Round 5: the leaf pass's second check with the normals as halves (8 B per entry: half the
# L2 traffic of its loads; measured 2 % slower, not kept): leaf-pass parity, boat vs HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05aj_pytest_parity.log 2>&1
rc=$?; tail -2 $P/r05aj_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/head/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 > $P/r05aj_ab_bp.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py ablib/head/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 >> $P/r05aj_ab_bp.log 2>&1
rc=$?; grep '"lib"' $P/r05aj_ab_bp.log; [ $rc -eq 0 ] || exit $rc

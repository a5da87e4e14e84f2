#!/bin/bash
# Round 5: the leaf pass's chunks with neighbours merged up to 16 entries (builder leaves of 16 or
# 8) against unmerged 16-entry leaves, boat in process; parity on the merged build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/m16_16/libpt_hip.so ablib/m8_16/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 > $P/r05ak_ab_merge.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py ablib/m8_16/libpt_hip.so ablib/m16_16/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 >> $P/r05ak_ab_merge.log 2>&1
rc=$?; grep '"lib"' $P/r05ak_ab_merge.log; [ $rc -eq 0 ] || exit $rc

#!/bin/bash
# Round 5: the leaf pass's chunk nodes loaded two ahead through the scalar cache (ablib/pf2) against
# one ahead, boat in process (no gain; not kept).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/pf2/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 > $P/r05aq_ab_pf2.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py ablib/pf2/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 >> $P/r05aq_ab_pf2.log 2>&1
rc=$?; grep '"lib"' $P/r05aq_ab_pf2.log; [ $rc -eq 0 ] || exit $rc

#!/bin/bash
# Round 5: the second check's normal loads without a branch per entry (clamped index; 7 % slower,
# not kept), unrolled by
# 2 / 4 / 8 (81 / 86 / 98 VGPRs), against HEAD's branchy loop (71 VGPRs, 7 waves); boat in process.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/bu2/libpt_hip.so ablib/bu4/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 > $P/r05ao_ab_refine_loads.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py ablib/bu4/libpt_hip.so ablib/bu2/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 >> $P/r05ao_ab_refine_loads.log 2>&1
rc=$?; grep '"lib"' $P/r05ao_ab_refine_loads.log; [ $rc -eq 0 ] || exit $rc

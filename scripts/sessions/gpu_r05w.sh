#!/bin/bash
# Round 5: with the second check the tests are cheap and the chunk checks are the cost: chunks of
# 16 / 24 entries (fewer checks) against 8, in process on the boat.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/chunk16/libpt_hip.so ablib/chunk24/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 > $P/r05w_ab_chunk_refine.log 2>&1
rc=$?; grep '"lib"' $P/r05w_ab_chunk_refine.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py ablib/chunk24/libpt_hip.so ablib/chunk16/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 >> $P/r05w_ab_chunk_refine.log 2>&1
rc=$?; grep '"lib"' $P/r05w_ab_chunk_refine.log | tail -3; [ $rc -eq 0 ] || exit $rc

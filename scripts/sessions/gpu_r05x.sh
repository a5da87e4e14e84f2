#!/bin/bash
# Round 5: chunks of 16 against 8 where the big leaves stay in the traversal (CornellBox2 with every
# mesh: AUTO keeps leaf_pre off there) and on the boat's SAH tree (its emitter leaf), in process.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
: > $P/r05x_ab_chunk16.log
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/chunk16/libpt_hip.so --scene CornellBox2 --all-meshes --res 1024 --spp 4 --depth 16 --rounds 3 >> $P/r05x_ab_chunk16.log 2>&1
rc=$?; grep '"lib"' $P/r05x_ab_chunk16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py ablib/chunk16/libpt_hip.so $L --scene CornellBox2 --all-meshes --res 1024 --spp 4 --depth 16 --rounds 3 >> $P/r05x_ab_chunk16.log 2>&1
rc=$?; grep '"lib"' $P/r05x_ab_chunk16.log | tail -2; [ $rc -eq 0 ] || exit $rc

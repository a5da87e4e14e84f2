#!/bin/bash
# Round 5: the round-4 library (6f469de) against the current one in process on the mailbox scenes
# (Mirror at depth 16, the bench's CornellBox at depth 8) and Glossy: did a round-5 change cost them?
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
: > $P/r05r_ab_r04.log
for args in "--scene CornellBox-Mirror --res 1024 --spp 64 --depth 16" "--scene CornellBox --res 1024 --spp 64 --depth 8" "--scene CornellBox-Glossy --res 1024 --spp 32 --depth 16"; do
  timeout -k 10 300 python3 scripts/ab_libs.py $L ablib/r04/libpt_hip.so $args --rounds 4 --async-torch >> $P/r05r_ab_r04.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $P/r05r_ab_r04.log; exit $rc; }
  timeout -k 10 300 python3 scripts/ab_libs.py ablib/r04/libpt_hip.so $L $args --rounds 4 --async-torch >> $P/r05r_ab_r04.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $P/r05r_ab_r04.log; exit $rc; }
done
grep '"lib"' $P/r05r_ab_r04.log

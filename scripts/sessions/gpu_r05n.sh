#!/bin/bash
# Round 5: leaf chunks of 16 / 12 entries against 8 (the pair walk's checks vs tests), in process on
# the boat; the boat's configs[3] line at the current head.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/chunk16/libpt_hip.so ablib/chunk12/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 3 > $P/r05n_ab_chunk.log 2>&1
rc=$?; grep lib $P/r05n_ab_chunk.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene MedievalBoat --width 1920 --height 1080 --spp 512 --depth 16 > $P/r05n_boat.log 2>&1
rc=$?; grep '^{' $P/r05n_boat.log > $P/r05n_boat.json; cat $P/r05n_boat.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc

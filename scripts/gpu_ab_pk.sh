#!/bin/bash
# in-process A/B: default build vs phase 1 in packed entry pairs (ablib/pk: extension instances,
# ablib/pk2: both instances), CornellBox 1024^2 64 spp depth 8, both orders
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 300 python3 scripts/ab_libs.py $B ablib/pk/libpt_hip.so ablib/pk2/libpt_hip.so --async-torch --rounds 5 > gpurun_out/ab_pk1.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_libs.py ablib/pk2/libpt_hip.so ablib/pk/libpt_hip.so $B --async-torch --rounds 5 > gpurun_out/ab_pk2.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_libs.py $B ablib/pk2/libpt_hip.so --async-torch --rounds 5 --scene CornellBox-Mirror --depth 16 > gpurun_out/ab_pk3.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_pk*.log

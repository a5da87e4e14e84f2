#!/bin/bash
# Round 6: phase 1 with the next entry's record in flight (PT_P1_PREFETCH=1 build) against the tree.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
P=ablib/p1pf/libpt_hip.so
timeout -k 10 400 python -u scripts/ab_libs.py $L $P $L $P --rounds 5 --async-torch --scene CornellBox --res 1024 --spp 64 --depth 8 > gpurun_out/r06v_ab_cornell.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/ab_libs.py $L $P --rounds 5 --async-torch --scene CornellBox-Mirror --res 1024 --spp 64 --depth 16 > gpurun_out/r06v_ab_mirror.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06v_ab_*.log

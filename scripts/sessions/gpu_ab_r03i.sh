#!/bin/bash
# In-process A/B: the current build against ablib/r03i (the tree of commit 3aa137a, built with
# make OUT_DIR=...), both orders -> gpurun_out/ab_r03i*.log (box-to-box spread vs a regression)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 300 python3 scripts/ab_libs.py $B ablib/r03i/libpt_hip.so --async-torch --rounds 5 > gpurun_out/ab_r03i1.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_libs.py ablib/r03i/libpt_hip.so $B --async-torch --rounds 5 > gpurun_out/ab_r03i2.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_r03i*.log

#!/bin/bash
# in-process A/B: default vs phase-1 records read from LDS (ablib/ldsrec), packed pairs (ablib/pk3), both (ablib/ldspk)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 300 python3 scripts/ab_libs.py $B ablib/ldsrec/libpt_hip.so ablib/pk3/libpt_hip.so ablib/ldspk/libpt_hip.so --async-torch --rounds 5 > gpurun_out/ab_ldsrec1.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_libs.py ablib/ldspk/libpt_hip.so ablib/pk3/libpt_hip.so ablib/ldsrec/libpt_hip.so $B --async-torch --rounds 5 > gpurun_out/ab_ldsrec2.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_ldsrec*.log

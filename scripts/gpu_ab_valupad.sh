#!/bin/bash
# Injection A/B: the fused kernel with 16 extra VALU instructions per phase-1 entry
# (ablib/pad16: v_fmac a,b,b; pad16k1: v_fma_f32 with three sources; pad16k2: v_fmac a,b,c;
# pad16k3: v_add_u32 — make EXTRA="-DPT_DIAG_VALU_PAD=16 -DPT_DIAG_VALU_KIND=k" OUT_DIR=...) against
# the default build, in one process, both orders -> gpurun_out/ab_valupad*.log
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
L="ablib/pad16/libpt_hip.so ablib/pad16k1/libpt_hip.so ablib/pad16k2/libpt_hip.so ablib/pad16k3/libpt_hip.so"
R="ablib/pad16k3/libpt_hip.so ablib/pad16k2/libpt_hip.so ablib/pad16k1/libpt_hip.so ablib/pad16/libpt_hip.so"
timeout -k 10 300 python3 scripts/ab_libs.py $B $L --async-torch --rounds 5 > gpurun_out/ab_valupad1.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_libs.py $R $B --async-torch --rounds 5 > gpurun_out/ab_valupad2.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_valupad*.log

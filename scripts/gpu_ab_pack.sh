#!/bin/bash
# in-process A/B: the fused kernel's packed 88 B shadow entries (this tree) vs the 104 B layout
# (ablib/base = the tree before), CornellBox 1024^2 64 spp depth 8 and Mirror depth 16, both orders
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 300 python3 scripts/ab_libs.py ablib/base/libpt_hip.so $B --async-torch --rounds 7 > gpurun_out/ab_pack1.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_libs.py $B ablib/base/libpt_hip.so --async-torch --rounds 7 > gpurun_out/ab_pack2.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_libs.py ablib/base/libpt_hip.so $B --async-torch --rounds 5 --scene CornellBox-Mirror --depth 16 > gpurun_out/ab_pack3.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_pack*.log

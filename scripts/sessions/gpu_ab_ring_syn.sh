#!/bin/bash
# In-process A/B on the 100k-triangle synthetic scene: current build (auto ring / ring forced to 128)
# against ablib/r03j -> gpurun_out/ab_ring_syn*.log
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 400 python3 scripts/ab_libs.py $B ablib/noocc/libpt_hip.so ablib/r03j/libpt_hip.so --async-torch --rounds 3 --scene synthetic-100000 --depth 8 --spp 8 > gpurun_out/ab_ring_syn1.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_ring_syn*.log

#!/bin/bash
# cost of the boat's cooperative big-leaf turns: the product vs a diagnostic build whose turns test
# every big leaf twice (same images; the extra time is one pass); with leaf chunks on and off
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 400 python3 scripts/ab_libs.py $L ablib/bigx2/libpt_hip.so --scene MedievalBoat --res 1024 --spp 8 --depth 16 --rounds 3 > gpurun_out/ab_bigleaf.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_bigleaf.log

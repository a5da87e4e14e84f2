#!/bin/bash
# In-process A/B of k_wf_trace's hit ring (make EXTRA=-DPT_HIT_RING=64 OUT_DIR=../../ablib/ring64):
# a 64-entry ring (two windows) cuts 4 KB of LDS per 512-thread block: Glossy fits 4 blocks per CU (8 waves per SIMD)
# instead of 3 -> gpurun_out/ab_ring_*.log
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
for sc in "CornellBox-Glossy --depth 16 --spp 32" "MedievalBoat --res 512 --depth 16 --spp 16"; do
  n=$(echo $sc | cut -d' ' -f1)
  timeout -k 10 400 python3 scripts/ab_libs.py $B ablib/ring64/libpt_hip.so --async-torch --rounds 3 --scene $sc > gpurun_out/ab_ring_${n}_1.log 2>&1 || exit $?
  timeout -k 10 400 python3 scripts/ab_libs.py ablib/ring64/libpt_hip.so $B --async-torch --rounds 3 --scene $sc > gpurun_out/ab_ring_${n}_2.log 2>&1 || exit $?
done
grep -h '^{' gpurun_out/ab_ring_*.log

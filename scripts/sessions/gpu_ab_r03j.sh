#!/bin/bash
# In-process A/B: the current build against ablib/r03j (the tree of commit 5ab4030, before the
# adaptive hit ring; make OUT_DIR=...), both orders, on traversal scenes -> gpurun_out/ab_r03j_*.log
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
for sc in "synthetic-100000 --depth 8 --spp 8" "synthetic-1000000 --depth 8 --spp 4" "CornellBox-Glossy --depth 16 --spp 16" "MedievalBoat --res 512 --depth 16 --spp 16"; do
  n=$(echo $sc | cut -d' ' -f1)
  timeout -k 10 400 python3 scripts/ab_libs.py $B ablib/r03j/libpt_hip.so --async-torch --rounds 3 --scene $sc > gpurun_out/ab_r03j_${n}_1.log 2>&1 || exit $?
  timeout -k 10 400 python3 scripts/ab_libs.py ablib/r03j/libpt_hip.so $B --async-torch --rounds 3 --scene $sc > gpurun_out/ab_r03j_${n}_2.log 2>&1 || exit $?
done
grep -h '^{' gpurun_out/ab_r03j_*.log

#!/bin/bash
# Round 4: Glossy's leaves (40-61 entries) — with cooperative turns forced onto them (big_leaf=20),
# how many lanes of a wave wait at the same leaf when a turn starts?  (The diagnostic build's
# counters minus the product's, scripts/build_park_diag.sh.)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
P=gpurun_out/profiles/r04n_park_glossy.log
: > $P
for bl in 20 32; do
  echo "== CornellBox-Glossy 1024 4 spp depth 16, big_leaf=$bl" >> $P
  timeout -k 10 300 python3 scripts/ab_libs.py "$L@big_leaf=$bl" "ablib/parkdiag/libpt_hip.so@big_leaf=$bl" --scene CornellBox-Glossy --res 1024 --spp 4 --depth 16 --rounds 1 --counters >> $P 2>&1
  rc=$?; echo "park glossy $bl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -v amdgpu.ids $P

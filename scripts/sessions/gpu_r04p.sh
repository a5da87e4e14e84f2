#!/bin/bash
# Round 4: batch the parked lanes before a shared chunk walk — a turn starts only when at least
# PB lanes are parked (or no lane has anything else to do), so each walk serves more rays
# (ablib/pb4, pb8, pb16) — against main (a walk as soon as one lane parks).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04p_ab_parkbatch.log
: > $AB
ab() {
  for order in "$L ablib/pb4/libpt_hip.so ablib/pb8/libpt_hip.so ablib/pb16/libpt_hip.so" "ablib/pb16/libpt_hip.so ablib/pb8/libpt_hip.so ablib/pb4/libpt_hip.so $L"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 5 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
ab --scene synthetic-1000000 --res 1024 --spp 2 --depth 8
grep -v "^ *$" $AB | grep -v amdgpu.ids

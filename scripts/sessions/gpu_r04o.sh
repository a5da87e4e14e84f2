#!/bin/bash
# Round 4: the trace kernel capped at 6 waves per SIMD (ablib/w6: amdgpu_waves_per_eu(6); the shared chunk walk's instance 102 -> 80 VGPRs with 56 B of scratch spills) against main (4 waves on the boat) and the build before the chunk-walk changes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04o_ab_chunkwalk.log
: > $AB
ab() {
  for order in "ablib/head/libpt_hip.so $L ablib/w6/libpt_hip.so" "ablib/w6/libpt_hip.so $L ablib/head/libpt_hip.so"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 5 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
ab --scene synthetic-1000000 --res 1024 --spp 2 --depth 8
grep -v "^ *$" $AB | grep -v amdgpu.ids
true

ab --scene CornellBox-Glossy --res 1024 --spp 16 --depth 16
grep -v "^ *$" $AB | grep -v amdgpu.ids | tail -6

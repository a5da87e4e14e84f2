#!/bin/bash
# Round 4: several rays per big-leaf chunk walk (ablib/cmulti: chunk_turn_multi, up to 16 parked lanes at one leaf share the walk; 102 VGPRs) against main and the build before the chunk-walk changes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04i_ab_chunkwalk.log
: > $AB
ab() {
  for order in "ablib/head/libpt_hip.so $L ablib/cmulti/libpt_hip.so" "ablib/cmulti/libpt_hip.so $L ablib/head/libpt_hip.so"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 5 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
ab --scene synthetic-1000000 --res 1024 --spp 2 --depth 8
grep -v "^ *$" $AB | grep -v amdgpu.ids
true


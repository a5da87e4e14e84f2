#!/bin/bash
# Round 4: pooled leaf turns with runs of 2, 3 and 6 entries (ablib/run2, run3, run6) against main (runs of 4).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04aa_ab_run.log
: > $AB
ab() {
  for order in "$L ablib/run2/libpt_hip.so ablib/run3/libpt_hip.so ablib/run6/libpt_hip.so" "ablib/run6/libpt_hip.so ablib/run3/libpt_hip.so ablib/run2/libpt_hip.so $L"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 3 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene CornellBox-Glossy --res 1024 --spp 16 --depth 16
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8
ab --scene synthetic-12500 --res 1024 --spp 8 --depth 8
ab --scene synthetic-100000 --res 1024 --spp 4 --depth 8
ab --scene synthetic-1000000 --res 1024 --spp 2 --depth 8
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
grep -v "^ *$" $AB | grep -v amdgpu.ids
grep -v "^ *$" $AB | grep -v amdgpu.ids

#!/bin/bash
# Round 4: pooled leaf turns at the sweep's batch sizes — the 16-spp sweep line of the 1M scene came
# out below round 4's earlier one — main with leaf_pool=0 / 1 in process, both orders.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04x_ab_pool_spp.log
: > $AB
ab() {
  for order in "$L@leaf_pool=0 $L@leaf_pool=1" "$L@leaf_pool=1 $L@leaf_pool=0"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 3 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene synthetic-1000000 --res 1024 --spp 16 --depth 8
ab --scene synthetic-1000000 --res 1024 --spp 2 --depth 8
ab --scene synthetic-100000 --res 1024 --spp 16 --depth 8
ab --scene CornellBox-Glossy --res 1024 --spp 64 --depth 16
grep -v "^ *$" $AB | grep -v amdgpu.ids

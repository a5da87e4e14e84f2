#!/bin/bash
# Round 4: the lean traversal's turn policy with pooled leaf turns — node bias 1, 2, 3 against the
# default 4 (a leaf turn when leaf lanes >= bias x node lanes), in process, both orders.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04z_ab_node_bias.log
: > $AB
ab() {
  for order in "$L@node_bias=4 $L@node_bias=3 $L@node_bias=2 $L@node_bias=1" "$L@node_bias=1 $L@node_bias=2 $L@node_bias=3 $L@node_bias=4"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 3 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8
ab --scene synthetic-100000 --res 1024 --spp 8 --depth 8
ab --scene synthetic-1000000 --res 1024 --spp 4 --depth 8
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
grep -v "^ *$" $AB | grep -v amdgpu.ids

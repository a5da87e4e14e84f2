#!/bin/bash
# Round 4: the leaf turn with the pairs' remaining entries pooled over the whole wave (ablib/pool:
# lean_leaf_pool; runs of 8 entries dealt one per lane, per-lane bests lowered into 64-bit LDS keys)
# against main (lean16: each leaf lane tests its own pair, K per turn) on the traversal scenes;
# runs of 4 and 16 entries (ablib/pool4, pool16).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04s_ab_pool.log
: > $AB
ab() {
  for order in "$L ablib/pool/libpt_hip.so ablib/pool4/libpt_hip.so ablib/pool16/libpt_hip.so" "ablib/pool16/libpt_hip.so ablib/pool4/libpt_hip.so ablib/pool/libpt_hip.so $L"; do
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
# the pooled turn's node bias (leaf turns when leaf lanes >= bias x node lanes; default 4)
P=ablib/pool/libpt_hip.so
for order in "$P@node_bias=4 $P@node_bias=8 $P@node_bias=2 $L" "$L $P@node_bias=2 $P@node_bias=8 $P@node_bias=4"; do
  echo "== Glossy node bias order: $order" >> $AB
  timeout -k 10 300 python3 scripts/ab_libs.py $order --scene CornellBox-Glossy --res 1024 --spp 16 --depth 16 --rounds 3 --async-torch >> $AB 2>&1
  rc=$?; echo "ab bias rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -v "^ *$" $AB | grep -v amdgpu.ids | tail -10

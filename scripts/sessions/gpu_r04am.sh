#!/bin/bash
# Round 4: pooled leaf turns on the fast SAH trees (leaves <= 8; off there by default since runs of 4
# cost Glossy 3.6 %) — now with runs of 2 and node bias 1 / 4, in process, same bits.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
OUT=gpurun_out/profiles/r04am_sah_pool.log
: > $OUT
run() {
  echo "== $*" >> $OUT
  timeout -k 10 300 python3 scripts/env_ab.py --bvh sah "$@" >> $OUT 2>&1
  rc=$?; echo "env_ab $2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
V="kernel=wavefront leaf_pool=1,pool_run=2 leaf_pool=1,pool_run=2,node_bias=1 leaf_pool=1,pool_run=4 node_bias=1"
run --scene CornellBox-Glossy --spp 64 --depth 16 --reps 3 $V
run --scene MedievalBoat --width 960 --height 960 --spp 32 --depth 16 --reps 3 $V
run --synthetic 100000 --spp 16 --depth 8 --reps 3 $V
run --synthetic 1000000 --spp 16 --depth 8 --reps 3 $V
grep -v "^ *$" $OUT | grep -v amdgpu.ids

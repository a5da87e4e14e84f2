#!/bin/bash
# Round 4: runs of 2 with node bias 1 / 2 on the scenes that default to runs of 4 (Glossy, the boat,
# the 1k and 12.5k synthetic trees), in process, both orders, same bits.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
OUT=gpurun_out/profiles/r04ak_run2_bias.log
: > $OUT
run() {
  echo "== $*" >> $OUT
  timeout -k 10 300 python3 scripts/env_ab.py "$@" >> $OUT 2>&1
  rc=$?; echo "env_ab $2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
V1="kernel=wavefront pool_run=2,node_bias=1 pool_run=2,node_bias=2 node_bias=1"
V2="node_bias=1 pool_run=2,node_bias=2 pool_run=2,node_bias=1 kernel=wavefront"
run --scene CornellBox-Glossy --spp 16 --depth 16 --reps 3 $V1
run --scene CornellBox-Glossy --spp 16 --depth 16 --reps 3 $V2
run --scene MedievalBoat --width 960 --height 960 --spp 8 --depth 16 --reps 3 $V1
run --scene MedievalBoat --width 960 --height 960 --spp 8 --depth 16 --reps 3 $V2
run --synthetic 12500 --spp 16 --depth 8 --reps 3 $V1
run --synthetic 12500 --spp 16 --depth 8 --reps 3 $V2
run --synthetic 1000 --spp 16 --depth 8 --reps 3 $V1
grep -v "^ *$" $OUT | grep -v amdgpu.ids

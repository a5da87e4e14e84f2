#!/bin/bash
# Round 4: the turn policy's node bias on the trees that pool runs of 2 (r04ah: node_bias=2 +3 %
# on 100k, +2 % on 1M), both orders, sweep configuration, in process, same bits.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
OUT=gpurun_out/profiles/r04ai_node_bias.log
: > $OUT
run() {
  echo "== $*" >> $OUT
  timeout -k 10 300 python3 scripts/env_ab.py "$@" >> $OUT 2>&1
  rc=$?; echo "env_ab $2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for N in 100000 1000000; do
  run --synthetic $N --spp 16 --depth 8 --reps 5 'node_bias=4' 'node_bias=3' 'node_bias=2' 'node_bias=1'
  run --synthetic $N --spp 16 --depth 8 --reps 5 'node_bias=1' 'node_bias=2' 'node_bias=3' 'node_bias=4'
done
run --synthetic 100000 --spp 4 --depth 8 --reps 5 'node_bias=4' 'node_bias=2' 'node_bias=4,pool_run=4' 'node_bias=2,pool_run=4'
grep -v "^ *$" $OUT | grep -v amdgpu.ids

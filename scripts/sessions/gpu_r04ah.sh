#!/bin/bash
# Round 4: the traversal kernel's tuning options re-checked on the large synthetic trees now that
# they pool runs of 2 (sweep configuration: 1024^2, 16 spp, depth 8), in process, same bits.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
OUT=gpurun_out/profiles/r04ah_env_ab.log
: > $OUT
run() {
  echo "== $*" >> $OUT
  timeout -k 10 300 python3 scripts/env_ab.py "$@" >> $OUT 2>&1
  rc=$?; echo "env_ab $1 $2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for N in 100000 1000000; do
  run --synthetic $N --spp 16 --depth 8 --reps 3 'pool_run=2' 'pool_run=4' 'node_bias=2' 'node_bias=8' 'sort=64' 'sort=0' 'trace_sparse=0' 'trace_sparse=8' 'big_leaf=64' 'trace_ring=128'
done
grep -v "^ *$" $OUT | grep -v amdgpu.ids

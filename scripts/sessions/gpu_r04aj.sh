#!/bin/bash
# Round 4: node bias 1 by default where leaf turns pool runs of 2 — parity and fast-tree suites,
# the default against node_bias=4 in process, then the BVH-size sweep with the final build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fast_trees.py tests/test_gpu_leafbvh.py > gpurun_out/profiles/r04aj_tests.log 2>&1
rc=$?; tail -1 gpurun_out/profiles/r04aj_tests.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/profiles/r04aj_default_vs_bias4.log
: > $OUT
for N in 100000 1000000; do
  echo "== synthetic $N" >> $OUT
  timeout -k 10 300 python3 scripts/env_ab.py --synthetic $N --spp 16 --depth 8 --reps 3 'kernel=wavefront' 'node_bias=4' >> $OUT 2>&1
  rc=$?; echo "env_ab $N rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep "variant" $OUT
timeout -k 10 900 bash scripts/gpu_sweep.sh r04aj
rc=$?; echo "sweep rc=$rc"; exit $rc

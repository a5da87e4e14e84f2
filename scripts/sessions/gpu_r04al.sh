#!/bin/bash
# Round 4 final build: runs of 2 (and node bias 1) where leaves reference >= 32 Ki triangles and no
# leaf is big — the GPU suite and smoke, the new default against runs of 4 / bias 4 on 12.5k and the
# boat (which keeps 4), then the BVH-size sweep.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/profiles/r04al_pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/profiles/r04al_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/profiles/r04al_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/profiles/r04al_smoke.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/profiles/r04al_default_ab.log
: > $OUT
for order in "kernel=wavefront pool_run=4,node_bias=4" "pool_run=4,node_bias=4 kernel=wavefront"; do
  echo "== synthetic 12500 $order" >> $OUT
  timeout -k 10 300 python3 scripts/env_ab.py --synthetic 12500 --spp 16 --depth 8 --reps 3 $order >> $OUT 2>&1
  rc=$?; echo "env_ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep "variant\|==" $OUT
timeout -k 10 900 bash scripts/gpu_sweep.sh r04al
rc=$?; echo "sweep rc=$rc"; exit $rc

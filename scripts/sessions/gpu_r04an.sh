#!/bin/bash
# Round 4 final build: pooled leaf turns on every tree, runs of 2 on the SAH trees — GPU suite,
# smoke, the default against leaf_pool=0 on the SAH trees, config lines, the BVH-size sweep.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/profiles/r04an_pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/profiles/r04an_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/profiles/r04an_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/profiles/r04an_smoke.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/profiles/r04an_sah_default.log
: > $OUT
run() {
  echo "== $*" >> $OUT
  timeout -k 10 300 python3 scripts/env_ab.py --bvh sah "$@" >> $OUT 2>&1
  rc=$?; echo "env_ab $2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run --scene CornellBox-Glossy --spp 64 --depth 16 --reps 3 kernel=wavefront leaf_pool=0
run --scene MedievalBoat --width 960 --height 960 --spp 32 --depth 16 --reps 3 kernel=wavefront leaf_pool=0
run --synthetic 12500 --spp 16 --depth 8 --reps 3 kernel=wavefront leaf_pool=0
run --synthetic 1000 --spp 16 --depth 8 --reps 3 kernel=wavefront leaf_pool=0
grep "variant\|==" $OUT
timeout -k 10 900 bash scripts/gpu_configs.sh r04an
rc=$?; echo "configs rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash scripts/gpu_sweep.sh r04an
rc=$?; echo "sweep rc=$rc"; exit $rc

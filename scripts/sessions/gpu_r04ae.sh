#!/bin/bash
# Round 4: pooled runs of 2 as their own k_wf_trace instances (template PRUN) against compile-time runs
# of 4 (ablib/base) and both runs inlined into one kernel (ablib/tmpl)
# then the parity and fast-tree suites on the new build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04ae_ab_runtime_run.log
: > $AB
ab() {
  for order in "$L ablib/base/libpt_hip.so ablib/tmpl/libpt_hip.so" "ablib/tmpl/libpt_hip.so ablib/base/libpt_hip.so $L"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 3 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fast_trees.py tests/test_gpu_leafbvh.py > gpurun_out/profiles/r04ae_tests.log 2>&1
rc=$?; tail -3 gpurun_out/profiles/r04ae_tests.log; [ $rc -eq 0 ] || exit $rc
ab --scene CornellBox-Glossy --res 1024 --spp 16 --depth 16
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
ab --scene synthetic-100000 --res 1024 --spp 4 --depth 8
ab --scene synthetic-1000000 --res 1024 --spp 2 --depth 8
grep -v "^ *$" $AB | grep -v amdgpu.ids

#!/bin/bash
# Round 4: the bench configuration (CornellBox 1024^2, 256 spp, depth 8: k_wf_step_bf) with this
# build against the build before the pooled run-length change (ablib/base, 59ad414), in process
# both orders — is r04af's 2690 Msamples/s the box or the code? — then the BVH-size sweep.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04ag_ab_bench.log
: > $AB
for order in "$L ablib/base/libpt_hip.so" "ablib/base/libpt_hip.so $L"; do
  echo "== CornellBox 1024 256spp D8 order: $order" >> $AB
  timeout -k 10 300 python3 scripts/ab_libs.py $order --scene CornellBox --res 1024 --spp 256 --depth 8 --rounds 5 --async-torch >> $AB 2>&1
  rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -v "^ *$" $AB | grep -v amdgpu.ids
timeout -k 10 900 bash scripts/gpu_sweep.sh r04ag
rc=$?; echo "sweep rc=$rc"; exit $rc

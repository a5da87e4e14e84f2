#!/bin/bash
# Round 4: the boat's chunk walk, latency.  main = branch-free chunk checks (the node's four loads
# issue together), the gathered chunks' permute merged one block later, DPP minima instead of
# ds_bpermute butterflies; ablib/cfull = main + the test pass's two records loaded together
# (86 VGPRs); ablib/head = the committed build before these.  Bits must match; then the parity
# tests of the leaf chunks.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04g_ab_chunkwalk.log
: > $AB
ab() {
  for order in "ablib/head/libpt_hip.so $L ablib/cfull/libpt_hip.so" "ablib/cfull/libpt_hip.so $L ablib/head/libpt_hip.so"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 5 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
ab --scene synthetic-1000000 --res 1024 --spp 2 --depth 8
ab --scene CornellBox-Glossy --res 1024 --spp 16 --depth 16
grep -v "^ *$" $AB | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread -k "leaf or boat or big or synthetic or fast_trees or config_bands" > gpurun_out/profiles/r04g_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/profiles/r04g_pytest_gpu.log

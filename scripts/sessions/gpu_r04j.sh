#!/bin/bash
# Round 4: the multi-ray chunk walk (main: chunk_turn_multi, up to 16 rays, checks and gathers in
# one loop, 102 VGPRs) against its two-phase form (ablib/m2: a block's checks for every ray first,
# the open masks kept as lanes of two registers, so the node's registers are free before a test
# pass: 91 VGPRs) and the same with up to 32 rays (ablib/m2x32), and the build before the
# chunk-walk changes (ablib/head).  Then the leaf-chunk tests (including the multi-ray self-test)
# and the parity tests that run the chunk walk.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04j_ab_multi.log
: > $AB
ab() {
  for order in "ablib/head/libpt_hip.so $L ablib/m2/libpt_hip.so ablib/m2x32/libpt_hip.so" "ablib/m2x32/libpt_hip.so ablib/m2/libpt_hip.so $L ablib/head/libpt_hip.so"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 5 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
grep -v "^ *$" $AB | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 600 --timeout-method thread -k "leaf or boat or big or synthetic or fast_trees or config_bands or kernel" > gpurun_out/profiles/r04j_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/profiles/r04j_pytest_gpu.log

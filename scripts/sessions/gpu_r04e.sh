#!/bin/bash
# Round 4: 16-bit stacks, second layout.  The paired layout (two levels per lane word) raised
# k_wf_trace's occupancy 6 -> 8 waves/SIMD on Glossy but issued +12 % VALU (r04d PMC); ablib/s16s
# keeps level k of lane i at u16 index k * lanes + i — the 32-bit stack's addressing at half the
# bytes.  In process against the product build with stack16 off and on (paired).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
S=ablib/s16s/libpt_hip.so
AB=gpurun_out/profiles/r04e_ab_stack16_layout.log
: > $AB
ab() {
  for order in "$L@stack16=0 $L@stack16=1 $S@stack16=1" "$S@stack16=1 $L@stack16=1 $L@stack16=0"; do
    echo "== $* order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order "$@" --rounds 5 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
ab --scene CornellBox-Glossy --res 1024 --spp 32 --depth 16
ab --scene MedievalBoat --res 960 --spp 8 --depth 16
ab --scene synthetic-1000 --res 1024 --spp 16 --depth 8
ab --scene synthetic-100000 --res 1024 --spp 8 --depth 8
grep -v "^ *$" $AB | grep -v amdgpu.ids
# verdict r03 item 3 step 3: lanes parked at the same big leaf per cooperative turn (the boat), from
# the diagnostic build's counters minus the product's (scripts/build_park_diag.sh)
P=gpurun_out/profiles/r04e_park_diag.log
: > $P
for sc in "--scene MedievalBoat --res 960 --spp 2 --depth 16" "--scene CornellBox-Glossy --res 1024 --spp 4 --depth 16"; do
  echo "== $sc" >> $P
  timeout -k 10 300 python3 scripts/ab_libs.py $L ablib/parkdiag/libpt_hip.so $sc --rounds 1 --counters >> $P 2>&1
  rc=$?; echo "park diag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -v amdgpu.ids $P
# cooperative turns for Glossy's medium leaves (largest 61 entries: never cooperative at the
# default threshold 128)
timeout -k 10 300 python3 scripts/env_ab.py --scene CornellBox-Glossy --spp 16 --depth 16 --reps 3 big_leaf=128 big_leaf=48 big_leaf=32 big_leaf=20 > gpurun_out/profiles/r04e_ab_glossy_bigleaf.jsonl 2>gpurun_out/ab.err
rc=$?; echo "glossy big_leaf rc=$rc"; cat gpurun_out/profiles/r04e_ab_glossy_bigleaf.jsonl; [ $rc -eq 0 ] || exit $rc

#!/bin/bash
# Round 4: parity suite on the reverted build (replay skips and div_r out), in-process A/B of the
# fused kernel's early exit of idle blocks (main = base + folded glass constants + early exit,
# ablib/noearly = main without it, ablib/base = the build before the round-4 kernel changes), and
# PMC passes on CornellBox-Glossy's trace kernel with 16-bit stacks on and off (resident waves,
# waits, LDS bank conflicts: why the occupancy step did not pay).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/profiles/r04d_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/profiles/r04d_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04d_ab_early.log
: > $AB
for sc in CornellBox CornellBox-Mirror; do
  for order in "$L ablib/noearly/libpt_hip.so ablib/base/libpt_hip.so" "ablib/base/libpt_hip.so ablib/noearly/libpt_hip.so $L"; do
    d=8; [ $sc = CornellBox-Mirror ] && d=16
    echo "== $sc depth $d order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order --scene $sc --res 1024 --spp 64 --depth $d --rounds 5 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $sc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
for order in "$L ablib/noearly/libpt_hip.so ablib/base/libpt_hip.so" "ablib/base/libpt_hip.so ablib/noearly/libpt_hip.so $L"; do
  echo "== CornellBox depth 8, 32 frames, order: $order" >> $AB
  timeout -k 10 300 python3 scripts/ab_libs.py $order --scene CornellBox --res 1024 --spp 32 --depth 8 --rounds 7 --async-torch >> $AB 2>&1
  rc=$?; echo "ab share rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -v "^ *$" $AB | grep -v amdgpu.ids
for s in 1 0; do
  OUT=gpurun_out/r04d_s16_$s
  mkdir -p $OUT
  CMD="python3 scripts/env_ab.py --scene CornellBox-Glossy --spp 8 --depth 16 --reps 1 stack16=$s"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $CMD > $OUT/kt.log 2>&1
  rc=$?; echo "stack16=$s kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1
    rc=$?; echo "stack16=$s pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/summarize_pmc.py $OUT k_wf_trace > gpurun_out/profiles/r04d_pmc_stack16_$s.txt 2>&1
  cat gpurun_out/profiles/r04d_pmc_stack16_$s.txt
done

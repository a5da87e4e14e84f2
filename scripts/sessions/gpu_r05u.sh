#!/bin/bash
# Round 5: kernel split and PMC of the leaf pass with the second check (HEAD) and without it
# (ablib/head), boat 960^2, 4 spp.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
for V in new head; do
  if [ $V = new ]; then L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so; else L=ablib/head/libpt_hip.so; fi
  OUT=gpurun_out/r05u_$V
  mkdir -p $OUT
  CMD="python3 scripts/ab_libs.py $L --scene MedievalBoat --res 960 --spp 4 --depth 16 --rounds 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $CMD > $OUT/kt.log 2>&1
  rc=$?; echo "$V kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=0
  for PM in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
            "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $PM --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1
    rc=$?; echo "$V pmc $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/summarize_pmc.py $OUT k_wf_leafpass k_wf_trace > $P/r05u_pmc_$V.txt 2>&1
done
head -24 $P/r05u_pmc_new.txt; head -24 $P/r05u_pmc_head.txt

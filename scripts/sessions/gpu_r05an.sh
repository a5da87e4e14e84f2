#!/bin/bash
# Round 5: PMC of the final library's leaf pass and traversal on the boat (960^2, 4 spp).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
OUT=gpurun_out/r05an
mkdir -p $OUT
CMD="python3 scripts/ab_libs.py brown-cs2240-path-tracer_amd/lib/libpt_hip.so --scene MedievalBoat --res 960 --spp 4 --depth 16 --rounds 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $CMD > $OUT/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for PM in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
          "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PM --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/summarize_pmc.py $OUT k_wf_leafpass k_wf_trace > $P/r05an_pmc_boat.txt 2>&1
cat $P/r05an_pmc_boat.txt

#!/bin/bash
# Round 5: the boat's render kernels under the same counters as round 4 (gpu_r04f.sh, before):
# k_wf_trace_pre (traversal with pre-resolved big leaves) and k_wf_leafpass, one kernel-trace
# pass and three PMC passes of the same command.  -> gpurun_out/profiles/r05f_*
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 300 python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 960 --spp 8 --depth 16 --reps 2 --profile 'parts=1' 'parts=1,leaf_pre=0' > gpurun_out/profiles/r05f_ab_parts1.log 2>&1
rc=$?; echo "parts=1 A/B rc=$rc"; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r05f_boat
mkdir -p $OUT
CMD="python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --spp 2 --depth 16 --reps 1 big_leaf=128"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $CMD > $OUT/kt.log 2>&1
rc=$?; echo "boat kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for P in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1
  rc=$?; echo "boat pmc pass $i rc=$rc"; tail -2 $OUT/pmc$i.log; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/summarize_pmc.py $OUT k_wf_trace k_wf_leafpass > gpurun_out/profiles/r05f_pmc_boat.txt 2>&1
cat gpurun_out/profiles/r05f_pmc_boat.txt

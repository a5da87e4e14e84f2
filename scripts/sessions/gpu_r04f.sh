#!/bin/bash
# Round 4: the GPU suite on the build without 16-bit stacks, then the boat's traversal kernel under
# L2 / L1 counters (is the big-leaf chunk walk bound by L2 bandwidth?): the counter list, one pass
# of TCC / TCP request counters and one of SQ issue counters.  -> gpurun_out/profiles/r04f_*
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/profiles/r04f_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/profiles/r04f_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 60 rocprofv3 -L > gpurun_out/profiles/r04f_counters_list.txt 2>&1; echo "counter list rc=$?"
OUT=gpurun_out/r04f_boat
mkdir -p $OUT
CMD="python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --spp 2 --depth 16 --reps 1 big_leaf=128"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $CMD > $OUT/kt.log 2>&1
rc=$?; echo "boat kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for P in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1
  rc=$?; echo "boat pmc pass $i rc=$rc"; tail -2 $OUT/pmc$i.log
done
python3 scripts/summarize_pmc.py $OUT k_wf_trace > gpurun_out/profiles/r04f_pmc_boat.txt 2>&1
cat gpurun_out/profiles/r04f_pmc_boat.txt

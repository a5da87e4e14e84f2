#!/bin/bash
# VALU issue calibration: pt_selftest_valu (peak VALU issue by construction) timed, then under a
# PMC pass of the same counters collect_traffic.sh reads for the render kernels; the constant of
# the valu_issue formula follows (scripts/calibrate_valu.py) -> gpurun_out/profiles/valu_calibration.json
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/valucal
rm -rf $OUT; mkdir -p $OUT gpurun_out/profiles
timeout -k 10 120 python3 scripts/calibrate_valu.py run --iters 20000 --reps 3 > $OUT/plain.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/calibrate_valu.py run --iters 20000 --reps 3 --packed >> $OUT/plain.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/calibrate_valu.py run --iters 20000 --reps 3 --mixed >> $OUT/plain.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/calibrate_valu.py run --iters 20000 --reps 3 --dep packed >> $OUT/plain.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/calibrate_valu.py run --iters 20000 --reps 3 --dep plain >> $OUT/plain.log 2>&1 || exit $?
cat $OUT/plain.log | grep '^{'
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/pmc -o run -- python3 scripts/calibrate_valu.py run --iters 20000 --reps 3 > $OUT/pmc.log 2>&1 || exit $?
python3 scripts/calibrate_valu.py summarize $OUT/pmc $OUT/pmc.log gpurun_out/profiles/valu_calibration.json || exit $?
# the same at the render kernel's dispatch length (~0.15 ms): does the formula hold on short dispatches?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/pmc_short -o run -- python3 scripts/calibrate_valu.py run --iters 320 --reps 40 > $OUT/pmc_short.log 2>&1 || exit $?
python3 scripts/calibrate_valu.py summarize $OUT/pmc_short $OUT/pmc_short.log gpurun_out/profiles/valu_calibration_short.json

#!/bin/bash
# Round 5: pair walk for batches of >= 32 rays and windows shrunk only below half the waves, against
# ablib/r05k; PMC of the leaf pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "big or leaf or nopre" > $P/r05l_pytest_parity.log 2>&1
rc=$?; tail -2 $P/r05l_pytest_parity.log; [ $rc -eq 0 ] || exit $rc
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 600 python3 scripts/ab_libs.py ablib/r05i/libpt_hip.so ablib/r05k/libpt_hip.so $L --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 > $P/r05l_ab_pairs.log 2>&1
rc=$?; grep lib $P/r05l_ab_pairs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/ab_libs.py $L ablib/r05k/libpt_hip.so ablib/r05i/libpt_hip.so --scene MedievalBoat --res 960 --spp 8 --depth 16 --rounds 4 >> $P/r05l_ab_pairs.log 2>&1
rc=$?; tail -3 $P/r05l_ab_pairs.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r05l_boat
mkdir -p $OUT
CMD="python3 scripts/env_ab.py --scene MedievalBoat --width 960 --height 540 --spp 2 --depth 16 --reps 1 big_leaf=128"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $CMD > $OUT/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for PM in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
          "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PM --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/summarize_pmc.py $OUT k_wf_leafpass k_wf_trace > $P/r05l_pmc_boat.txt 2>&1
cat $P/r05l_pmc_boat.txt

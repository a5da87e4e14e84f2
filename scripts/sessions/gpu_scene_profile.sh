#!/bin/bash
# rocprofv3 kernel-trace stats + PMC (VALU lanes, waits, FETCH/WRITE) of bench.py on one scene.
# usage: gpu_scene_profile.sh TAG bench-args...   (outputs under gpurun_out/TAG/)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $*"
timeout -k 10 300 python3 bench.py $ARGS --steps 2 --warmup 1 > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || exit $?
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || exit $?
done
grep -h '^{' $OUT/bench.log | cut -c1-300
python3 scripts/summarize_pmc.py $OUT > $OUT/summary.txt; head -60 $OUT/summary.txt

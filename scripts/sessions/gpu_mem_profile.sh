#!/bin/bash
# memory-path PMC of bench.py on one scene (TA / TCP / TCC): where traversal loads wait.
# usage: gpu_mem_profile.sh TAG bench-args...   (outputs under gpurun_out/TAG/)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $*"
i=0
for P in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum" \
         "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || exit $?
done
python3 scripts/summarize_pmc.py $OUT > $OUT/summary.txt; head -80 $OUT/summary.txt

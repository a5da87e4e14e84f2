#!/bin/bash
# GPU-box profiling: counter list, kernel trace + stats, PMC passes (each its own run; no
# --pmc combined with sys/runtime traces).  Usage: gpu_profile.sh <tag> [perf_variants args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-prof}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="python3 scripts/perf_variants.py --rounds 1 $*"
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $CMD > $OUT/kt.log 2>&1
rc=$?; echo "kernel-trace rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
find $OUT -name "*.csv" | head -20
exit 0

#!/bin/bash
# HBM traffic and VALU issue of the bench's render kernels from rocprofv3 PMC counters, collected
# as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE in SEPARATE passes (TCC
# slots), no trace domains mixed with --pmc, FETCH_SIZE doubled (gfx950 tallies 128-B requests
# at 64 B), both in KB; a third pass reads SQ_ACTIVE_INST_VALU / GRBM_GUI_ACTIVE for the VALU
# issue fraction.  Writes per-launch figures (keyed by WxHxsppxdepthxworld) to
# gpurun_out/profiles/traffic.json (copy it into profiles/ locally); raw CSVs stay under
# gpurun_out/traffic/.  Extra arguments go to bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/traffic
rm -rf $OUT
mkdir -p $OUT
ARGS="--steps 2 --warmup 0 --no-cpu-baseline $*"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/valu -o run -- python3 bench.py $ARGS > $OUT/valu.log 2>&1 || exit $?
mkdir -p gpurun_out/profiles
cp profiles/traffic.json gpurun_out/profiles/traffic.json 2>/dev/null || true
python3 scripts/summarize_traffic.py gpurun_out/profiles/traffic.json

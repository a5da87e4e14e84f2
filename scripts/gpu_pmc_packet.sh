#!/bin/bash
# PMC of the camera-ray trace launches: k_wf_trace (packet=0) vs k_wf_trace_pk (packet=1), Glossy
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for P in 0 1; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_pk$P -o run -- python3 bench.py --scene CornellBox-Glossy --spp 8 --depth 16 --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing --opt packet=$P > gpurun_out/pmc_pk$P.log 2>&1 || exit $?
done
echo "packet=0 (k_wf_trace, first dispatches = camera rays of the counted render, then the timed)"
python3 scripts/pmc_dispatch.py gpurun_out/pmc_pk0/run_counter_collection.csv "k_wf_trace<" 40
echo "packet=1 (k_wf_trace_pk)"
python3 scripts/pmc_dispatch.py gpurun_out/pmc_pk1/run_counter_collection.csv "k_wf_trace_pk<" 8

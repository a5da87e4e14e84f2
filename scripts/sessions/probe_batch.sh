#!/bin/bash
# A/B probe of the wavefront batch size (option wf_paths): one bench line per (config, size)
# -> gpurun_out/probe/summary.txt.  Usage: scripts/probe_batch.sh "<bench args>" size...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
args=$1; shift
for wp in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $args --opt wf_paths=$wp > gpurun_out/probe/run.log 2>&1 || { echo FAIL $args $wp; tail -5 gpurun_out/probe/run.log; exit 1; }
  v=$(grep -h '^{' gpurun_out/probe/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')
  echo "$args wf_paths=$wp -> $v" | tee -a gpurun_out/probe/summary.txt
done

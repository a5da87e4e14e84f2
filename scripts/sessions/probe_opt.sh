#!/bin/bash
# A/B probe of one library option: one bench line per (config, value), in the order given
# -> gpurun_out/probe/summary.txt.  Usage: scripts/probe_opt.sh "<bench args>" NAME value...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
args=$1; name=$2; shift 2
for v in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $args --opt $name=$v > gpurun_out/probe/run.log 2>&1 || { echo FAIL $args $name=$v; tail -5 gpurun_out/probe/run.log; exit 1; }
  r=$(grep -h '^{' gpurun_out/probe/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')
  echo "$args $name=$v -> $r" | tee -a gpurun_out/probe/summary.txt
done

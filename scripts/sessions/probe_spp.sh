#!/bin/bash
# Strong-scaling rehearsal on one GPU: the bench config at 256 / N spp (the frames one of N ranks
# renders per step), one line each -> gpurun_out/probe/summary.txt
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
for spp in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --spp $spp > gpurun_out/probe/run.log 2>&1 || { echo FAIL $spp; tail -5 gpurun_out/probe/run.log; exit 1; }
  r=$(grep -h '^{' gpurun_out/probe/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_busy_ms_per_step"])')
  echo "spp=$spp -> $r" | tee -a gpurun_out/probe/summary.txt
done

#!/bin/bash
# Round 6: a rank's 1/8 share timed over 40 steps (5 steps of 12.6 ms carry the first step's ramp
# and the last step's per-launch events, ~4 % of the share) against N = 1 over 10 steps; twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06y2_bench.jsonl
for rep in 1 2; do
  for s in "--steps 10 --warmup 2" "--share-of 8 --steps 40 --warmup 5" "--share-of 8 --steps 40 --warmup 5 --no-kernel-timing"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $s > gpurun_out/r06y2_run.log 2>&1 || exit $?
    python3 -c "import json,sys; j=json.loads([l for l in open('gpurun_out/r06y2_run.log') if l.startswith('{')][-1]); r=j['roofline'].get('render_ms_steps') or []; print(json.dumps({'rep': $rep, 'args': '$s', 'value': j['value'], 'ms': j['ms_per_step'], 'render_ms_median': sorted(r)[len(r)//2] if r else None}))" | tee -a gpurun_out/r06y2_bench.jsonl
  done
done

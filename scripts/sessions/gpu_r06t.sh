#!/bin/bash
# Round 6: wavefront batch size in the bench (option wf_paths): 64 M paths (default), 128 M, 256 M
# (the whole 256-frame step in one batch), alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06t_bench.jsonl
for rep in 1 2; do
  for v in "" "--opt wf_paths=134217728" "--opt wf_paths=268435456"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $v > gpurun_out/r06t_run.log 2>&1 || exit $?
    python3 -c "import json,sys; j=json.loads([l for l in open('gpurun_out/r06t_run.log') if l.startswith('{')][-1]); print(json.dumps({'rep': $rep, 'opt': '$v', 'value': j['value'], 'ms': j['ms_per_step']}))" | tee -a gpurun_out/r06t_bench.jsonl
  done
done

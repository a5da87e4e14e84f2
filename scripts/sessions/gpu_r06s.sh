#!/bin/bash
# Round 6: streaming regeneration (option regen=128) in the bench itself: N = 1 and a rank's 1/8 share,
# default and regen=128 alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06s_bench.jsonl
for rep in 1 2; do
  for v in "" "--opt regen=128"; do
    for s in "" "--share-of 8"; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline $s $v > gpurun_out/r06s_run.log 2>&1 || exit $?
      python3 -c "import json,sys; j=json.loads([l for l in open('gpurun_out/r06s_run.log') if l.startswith('{')][-1]); print(json.dumps({'rep': $rep, 'opt': '$v', 'share': '$s', 'value': j['value'], 'ms': j['ms_per_step']}))" | tee -a gpurun_out/r06s_bench.jsonl
    done
  done
done

#!/bin/bash
# Round 5: the bench with events in the last timed step only — N = 1 and the 1/8 share.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
OUT=$P/r05af_bench_lastevents.jsonl
: > $OUT
run() { timeout -k 10 300 python3 -u bench.py "$@" > gpurun_out/af.log 2>&1; rc=$?; grep '^{' gpurun_out/af.log >> $OUT; return $rc; }
run --steps 5 --warmup 1 --no-cpu-baseline && run --steps 5 --warmup 1 --share-of 8 --no-cpu-baseline && run --steps 5 --warmup 1 --share-of 4 --no-cpu-baseline
rc=$?
python3 - <<'PY'
import json
for l in open("gpurun_out/profiles/r05af_bench_lastevents.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(d["config"].get("share") and d["config"]["share"]["of"], d["value"], d["ms_per_step"], r["kernel_busy_ms_per_step"], r["launches_per_step"], r["frac"])
PY
exit $rc

#!/bin/bash
# Round 5: the 1/8 rank share of configs[1] against N = 1 without the bench's per-launch events
# (--no-kernel-timing), and with one part (parts=1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
OUT=$P/r05ae_share_events.jsonl
: > $OUT
run() { timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > gpurun_out/ae.log 2>&1; rc=$?; grep '^{' gpurun_out/ae.log >> $OUT; return $rc; }
run --steps 5 --warmup 1 --no-kernel-timing &&
run --steps 5 --warmup 1 --share-of 8 --no-kernel-timing &&
run --steps 5 --warmup 1 --share-of 8 --no-kernel-timing --opt parts=1 &&
run --steps 5 --warmup 1 --share-of 8 --no-kernel-timing --opt parts=3
rc=$?
python3 - <<'PY'
import json
for l in open("gpurun_out/profiles/r05ae_share_events.jsonl"):
    d = json.loads(l); print(d["config"].get("share") and d["config"]["share"]["of"], d["config"].get("options"), d["value"], d["ms_per_step"])
PY
exit $rc

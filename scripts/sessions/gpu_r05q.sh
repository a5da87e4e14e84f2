#!/bin/bash
# Round 5 measurement, part 2: configs[2..3] lines (reference and SAH trees), the BVH-size sweep,
# and the rank shares of configs[1] / configs[4] (readback now overlapped with the next render).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
bash scripts/gpu_configs.sh r05q || exit $?
bash scripts/gpu_sweep.sh r05q || exit $?
cp gpurun_out/r05q_sweep.jsonl gpurun_out/profiles/r05q_sweep.jsonl
OUT=gpurun_out/profiles/r05q_shares.jsonl bash scripts/gpu_shares.sh > gpurun_out/shares.log 2>&1
rc=$?; echo "shares rc=$rc"; python3 - <<'PY'
import json
for l in open("gpurun_out/profiles/r05q_shares.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["config"].get("share"), d["config"]["workload"][:40], d["value"])
PY
exit $rc

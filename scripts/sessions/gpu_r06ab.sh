#!/bin/bash
# Round 6: configs[4]'s per-GPU share (CornellBox 4096^2, 4096 spp over 8 ranks: 512 frames per rank)
# timed alone, and configs[1] beside it on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06ab_cfg4_share.jsonl
timeout -k 10 400 python -u bench.py --no-cpu-baseline --width 4096 --height 4096 --spp 4096 --share-of 8 --steps 3 --warmup 1 > gpurun_out/r06ab_run.log 2>&1 || exit $?
grep '^{' gpurun_out/r06ab_run.log | tail -1 >> gpurun_out/r06ab_cfg4_share.jsonl
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06ab_run.log 2>&1 || exit $?
grep '^{' gpurun_out/r06ab_run.log | tail -1 >> gpurun_out/r06ab_cfg4_share.jsonl
python3 -c "import json; [print(json.loads(l)['config']['workload'][:60], json.loads(l)['value']) for l in open('gpurun_out/r06ab_cfg4_share.jsonl')]"

#!/bin/bash
# Round 6: the GEN launch's count-slot memsets on the caller's stream before the fork (the second
# part no longer starts ~0.5 ms late) — in-process A/B against HEAD (H) at the bench size and a
# rank's 1/8 share; then the bench and the 1/8 share with the tree's library.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
H=ablib/head/libpt_hip.so
timeout -k 10 400 python -u scripts/ab_libs.py $H $L $H $L --rounds 5 --async-torch --scene CornellBox --res 1024 --spp 32 --depth 8 > gpurun_out/r06w_ab_share.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/ab_libs.py $H $L $H $L --rounds 3 --async-torch --scene CornellBox --res 1024 --spp 256 --depth 8 > gpurun_out/r06w_ab_n1.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r06w_ab_*.log
: > gpurun_out/r06w_bench.jsonl
for s in "" "--share-of 8" "" "--share-of 8"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $s > gpurun_out/r06w_run.log 2>&1 || exit $?
  python3 -c "import json,sys; j=json.loads([l for l in open('gpurun_out/r06w_run.log') if l.startswith('{')][-1]); print(json.dumps({'share': '$s', 'value': j['value'], 'ms': j['ms_per_step']}))" | tee -a gpurun_out/r06w_bench.jsonl
done

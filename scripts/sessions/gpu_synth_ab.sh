#!/bin/bash
# env A/B on the synthetic sweep scenes (one bench line per variant)
# usage: gpu_synth_ab.sh TAG "N1 N2 .." "ENV=V ENV=V" "ENV=V" ...   (X=0: the defaults)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; NS=$2; shift 2
OUT=gpurun_out/${TAG}.jsonl
: > $OUT
for N in $NS; do
  for V in "$@"; do
    env $V timeout -k 10 300 python3 bench.py --synthetic $N --spp 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/syn.log 2>&1
    rc=$?; [ $rc -eq 0 ] || exit $rc
    echo "N=$N $V $(grep -h '^{' gpurun_out/syn.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')" | tee -a $OUT
  done
done

#!/bin/bash
# BVH-size sweep: synthetic Cornell-sized scenes of N triangles, the reference's
# builder and the fast SAH builder, one bench line each -> gpurun_out/<TAG>_sweep.jsonl
# usage: gpu_sweep.sh [TAG] [--gpus N ...]  (several --gpus: one line per N; N > 1 runs N ranks,
# bench.py launches them itself; north_star asks for 1, 2, 4 and 8 GPUs)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=r02
GPUS=""
while [ $# -gt 0 ]; do
  case "$1" in
    --gpus) GPUS="$GPUS $2"; shift 2 ;;
    *) TAG=$1; shift ;;
  esac
done
GPUS=${GPUS:-1}
SPP=${SPP:-16}
OUT=gpurun_out/${TAG}_sweep.jsonl
: > $OUT
for G in $GPUS; do
 for N in 36 1000 12500 100000 1000000; do
  for B in reference sah; do
    timeout -k 10 300 python3 bench.py --gpus $G --synthetic $N --bvh $B --spp $SPP --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_${N}_${B}_${G}.log 2>&1
    rc=$?; echo "gpus=$G N=$N bvh=$B rc=$rc"; [ $rc -eq 0 ] || exit $rc
    grep -h '^{' gpurun_out/sweep_${N}_${B}_${G}.log >> $OUT
  done
 done
done
python3 - "$OUT" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(d["n_gpus"], "GPU", d["config"]["scene_triangles"], d["config"]["bvh"], d["value"], "Msamples/s", r["kernel"], "frac", r["frac"])
PY

#!/bin/bash
# BVH-size sweep: synthetic Cornell-sized scenes of N triangles, the reference's
# builder and the fast SAH builder, one bench line each -> gpurun_out/<TAG>_sweep.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r02}
SPP=${SPP:-16}
OUT=gpurun_out/${TAG}_sweep.jsonl
: > $OUT
for N in 36 1000 12500 100000 1000000; do
  for B in reference sah; do
    timeout -k 10 300 python3 bench.py --synthetic $N --bvh $B --spp $SPP --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_${N}_${B}.log 2>&1
    rc=$?; echo "N=$N bvh=$B rc=$rc"; [ $rc -eq 0 ] || exit $rc
    grep -h '^{' gpurun_out/sweep_${N}_${B}.log >> $OUT
  done
done
python3 - "$OUT" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(d["config"]["scene_triangles"], d["config"]["bvh"], d["value"], "Msamples/s", r["kernel"], "frac", r["frac"])
PY

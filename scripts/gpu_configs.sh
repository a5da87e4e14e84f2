#!/bin/bash
# BASELINE.json configs[2..3] at their stated spp (depth 16, the reference default) plus the fast
# SAH tree of the same scenes: one bench line each -> gpurun_out/profiles/<TAG>_configs.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/profiles/${TAG}_configs.jsonl
mkdir -p gpurun_out/profiles
: > $OUT
run() {
  timeout -k 10 600 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/cfg.log 2>&1
  rc=$?; echo "config $* rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -h '^{' gpurun_out/cfg.log >> $OUT
}
run --scene CornellBox-Mirror --spp 1024 --depth 16
run --scene CornellBox-Glossy --spp 1024 --depth 16
run --scene CornellBox-Glossy --spp 1024 --depth 16 --bvh sah
run --scene MedievalBoat --width 1920 --height 1080 --spp 512 --depth 16
run --scene MedievalBoat --width 1920 --height 1080 --spp 512 --depth 16 --bvh sah
python3 - "$OUT" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(d["metric"], d["config"]["bvh"], d["value"], "Msamples/s", r["kernel"], "frac", r["frac"])
PY

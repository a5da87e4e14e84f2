#!/bin/bash
# BASELINE.json configs 3 and 4 (other scenes) at reduced spp: one bench line each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/configs.jsonl
: > $OUT
for args in "--scene CornellBox-Mirror --spp 64 --depth 16" "--scene CornellBox-Glossy --spp 64 --depth 16" \
            "--scene MedievalBoat --width 1920 --height 1080 --spp 16 --depth 16"; do
  timeout -k 10 300 python bench.py $args --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/cfg.log; exit $rc; fi
  grep "^{" gpurun_out/cfg.log >> $OUT
done
python3 -c "
import json
for l in open('$OUT'):
    d=json.loads(l); r=d['roofline']; print(d['config']['workload'], d['value'], r['kernel'], r.get('kernels_ms_warmup_step'))"

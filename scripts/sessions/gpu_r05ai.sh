#!/bin/bash
# Round 5: the boat's configs[3] line with the latest library (second check's terms by ds_bpermute).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/profiles
mkdir -p $P
timeout -k 10 600 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene MedievalBoat --width 1920 --height 1080 --spp 512 --depth 16 > $P/r05ai_boat.log 2>&1
rc=$?; grep '^{' $P/r05ai_boat.log > $P/r05ai_boat.json; python3 -c "
import json; d=json.loads(open('$P/r05ai_boat.json').read()); r=d['roofline']; print(d['value'], r['kernels_ms_warmup_step'])"; exit $rc

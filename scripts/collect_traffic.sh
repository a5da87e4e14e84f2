#!/bin/bash
# HBM traffic of the bench's render kernel from rocprofv3 PMC counters, collected as
# MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE in SEPARATE passes (TCC
# slots), no trace domains mixed with --pmc, FETCH_SIZE doubled (gfx950 tallies 128-B
# requests at 64 B), both in KB.  Writes profiles/traffic.json (per launch, keyed by
# WxHxsppxdepthxworld) and keeps the raw CSVs under gpurun_out/traffic/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/traffic
mkdir -p $OUT profiles
ARGS="--steps 2 --warmup 0 --no-cpu-baseline $*"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit $?
python3 - "$@" <<'PY'
import csv, glob, json, os, sys, collections
def load(tag, counter):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/traffic/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                agg[(r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (k, d), v in agg.items():
        per[k].append(sum(v))
    return {k: sum(v) / len(v) for k, v in per.items()}
fetch, write = load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
line = [json.loads(l) for l in open("gpurun_out/traffic/fetch.log") if l.startswith("{")][0]
cfg = line["config"]
W, H = 1024, 1024
import re
m = re.search(r"(\d+)x(\d+) (\d+)spp depth (\d+)", cfg["workload"])
key = f"{m.group(1)}x{m.group(2)}x{m.group(3)}x{m.group(4)}x{line['n_gpus']}"
path = "profiles/traffic.json"
t = json.load(open(path)) if os.path.exists(path) else {}
t[key] = {}
for k in fetch:
    short = k.split("::")[-1]
    fb, wb = fetch[k] * 1024 * 2, write.get(k, 0.0) * 1024
    t[key][short] = {"fetch_kb_raw": fetch[k], "write_kb": write.get(k, 0.0), "hbm_bytes_per_launch": fb + wb,
                     "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KB -> bytes, mean per dispatch"}
json.dump(t, open(path, "w"), indent=1)
print(json.dumps(t[key], indent=1))
PY

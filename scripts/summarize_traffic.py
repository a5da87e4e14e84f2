#!/usr/bin/env python3
"""Summarize rocprofv3 FETCH_SIZE / WRITE_SIZE passes (gpurun_out/traffic) into traffic.json.
Usage: summarize_traffic.py [out.json]"""
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
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}
(fetch, ndisp), (write, _) = load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
line = [json.loads(l) for l in open("gpurun_out/traffic/fetch.log") if l.startswith("{")][0]
cfg = line["config"]
W, H = 1024, 1024
import re
m = re.search(r"(\d+)x(\d+) (\d+)spp depth (\d+)", cfg["workload"])
key = f"{m.group(1)}x{m.group(2)}x{m.group(3)}x{m.group(4)}x{line['n_gpus']}"
path = sys.argv[1] if len(sys.argv) > 1 else "profiles/traffic.json"
t = json.load(open(path)) if os.path.exists(path) else {}
t[key] = {}
for k in fetch:
    short = k.split("::")[-1]
    fb, wb = fetch[k] * 1024 * 2, write.get(k, 0.0) * 1024
    t[key][short] = {"fetch_kb_raw": fetch[k], "write_kb": write.get(k, 0.0), "hbm_bytes_per_launch": fb + wb,
                     "dispatches": ndisp[k],
                     "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KB -> bytes, mean per dispatch"}
json.dump(t, open(path, "w"), indent=1)
print(json.dumps(t[key], indent=1))

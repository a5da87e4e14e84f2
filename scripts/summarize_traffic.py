#!/usr/bin/env python3
"""Summarize the rocprofv3 PMC passes of scripts/collect_traffic.sh (gpurun_out/traffic/{fetch,
write,valu}) into traffic.json: per kernel instance and launch, HBM bytes (FETCH_SIZE x 2 for
gfx950 + WRITE_SIZE, KB -> bytes) and the VALU issue fraction
    valu_issue = k * SQ_ACTIVE_INST_VALU / (128 * GRBM_GUI_ACTIVE)
(GRBM_GUI_ACTIVE summed over the 8 XCDs, each of 32 CUs x 4 SIMDs: SIMD-cycles = GRBM / 8 x 1024),
with k calibrated on a kernel that issues VALU at the SIMDs' peak by construction
(profiles/valu_calibration.json, scripts/calibrate_valu.sh: that kernel reads 1.0).  Without the
calibration file k = 4 (the uncalibrated quad-cycle reading, marked as such).
PMC passes serialise the kernels, so these are per-launch figures of a kernel running alone.
Usage: summarize_traffic.py [out.json]"""
import collections
import csv
import glob
import json
import os
import re
import sys

SRC = "gpurun_out/traffic"


def load(tag, counters):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{SRC}/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] in counters:
                # (anonymous-namespace kernels, e.g. k_wf_leafpass: drop the namespace before the cut at "(")
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
                k = (name.split("(")[0].replace("void ", ""), r["Dispatch_Id"])
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in agg.items():
        for n, v in cs.items():
            per[k][n].append(v)
    mean = {k: {n: sum(v) / len(v) for n, v in cs.items()} for k, cs in per.items()}
    ndisp = {k: max(len(v) for v in cs.values()) for k, cs in per.items()}
    return mean, ndisp


def calibration():
    path = "profiles/valu_calibration.json"
    try:
        c = json.load(open(path))
        return c["k_active"], f"{path} (k = {c['k_active']:.3f}: pt_selftest_valu reads 1.0)"
    except (OSError, KeyError, ValueError):
        return 4.0, "uncalibrated (k = 4, quad-cycle reading)"


def main():
    k_valu, cal_src = calibration()
    fetch, ndisp = load("fetch", {"FETCH_SIZE"})
    write, _ = load("write", {"WRITE_SIZE"})
    valu, _ = load("valu", {"SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_WAVE_CYCLES",
                            "SQ_WAVES", "GRBM_GUI_ACTIVE"})
    line = [json.loads(x) for x in open(f"{SRC}/fetch.log") if x.startswith("{")][0]
    m = re.search(r"(\d+)x(\d+) (\d+)spp depth (\d+)", line["config"]["workload"])
    key = f"{m.group(1)}x{m.group(2)}x{m.group(3)}x{m.group(4)}x{line['n_gpus']}"
    # the same entry under a key that names the scene and tree too (bench.py reads this one first: the
    # plain key is shared by every scene rendered at the same size, spp and depth)
    scene = line["config"]["workload"].split(".xml")[0]
    qkey = f"{scene}|{line['config'].get('bvh', 'reference')}|{key}"
    path = sys.argv[1] if len(sys.argv) > 1 else "profiles/traffic.json"
    t = json.load(open(path)) if os.path.exists(path) else {}
    t[key] = {"_source": "scripts/collect_traffic.sh: rocprofv3 --pmc passes FETCH_SIZE | WRITE_SIZE | SQ_ACTIVE_INST_VALU.. "
                         "GRBM_GUI_ACTIVE of `bench.py " + " ".join(sys.argv[2:]) + "` (" + line["config"]["workload"] + ")"}
    for k in fetch:
        short = k.split("::")[-1]
        fb, wb = fetch[k]["FETCH_SIZE"] * 1024 * 2, write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        e = {"fetch_kb_raw": fetch[k]["FETCH_SIZE"], "write_kb": write.get(k, {}).get("WRITE_SIZE", 0.0),
             "hbm_bytes_per_launch": fb + wb, "dispatches": ndisp[k],
             "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KB -> bytes, mean per dispatch"}
        v = valu.get(k)
        if v and v.get("GRBM_GUI_ACTIVE"):
            e["valu_issue"] = k_valu * v["SQ_ACTIVE_INST_VALU"] / (128.0 * v["GRBM_GUI_ACTIVE"])
            e["valu_issue_calibration"] = cal_src
            e["valu_lane_util"] = v.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * v["SQ_ACTIVE_INST_VALU"]) if v.get("SQ_ACTIVE_INST_VALU") else None
            e["valu_counters"] = v
        t[key][short] = e
    t[qkey] = t[key]
    json.dump(t, open(path, "w"), indent=1)
    print(json.dumps(t[key], indent=1))


if __name__ == "__main__":
    main()

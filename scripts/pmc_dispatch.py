#!/usr/bin/env python3
"""Per-dispatch PMC figures of one kernel family from a rocprofv3 --pmc counter CSV: VALU
wave-instructions, lane utilisation (SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)) and the
calibrated issue fraction, for the first dispatches (launch 0 of each batch part = camera rays).
usage: pmc_dispatch.py COUNTER_CSV KERNEL_PREFIX [n_first]"""
import collections
import csv
import json
import os
import sys

rows = collections.defaultdict(dict)
names = {}
for d in csv.DictReader(open(sys.argv[1])):
    name = d["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
    if not name.startswith(sys.argv[2]):
        continue
    k = int(d["Dispatch_Id"])
    rows[k][d["Counter_Name"]] = rows[k].get(d["Counter_Name"], 0.0) + float(d["Counter_Value"])
    names[k] = name
cal = 4.2
try:
    cal = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "valu_calibration.json")))["k_active"]
except (OSError, KeyError, ValueError):
    pass
n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
for k in sorted(rows)[:n]:
    c = rows[k]
    act = c.get("SQ_ACTIVE_INST_VALU", 0.0)
    out = {"dispatch": k, "kernel": names[k], "valu_wave_instr": c.get("SQ_INSTS_VALU"),
           "lane_util": round(c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * act), 4) if act else None,
           "valu_issue": round(cal * act / (128.0 * c["GRBM_GUI_ACTIVE"]), 4) if c.get("GRBM_GUI_ACTIVE") else None,
           "grbm_gui_active": c.get("GRBM_GUI_ACTIVE")}
    print(json.dumps(out))

#!/usr/bin/env python3
"""Per-launch durations of the render kernels from a rocprofv3 --kernel-trace CSV: which bounce
(launch index within a batch part) costs what.  usage: launch_profile.py KERNEL_TRACE_CSV [prefix]"""
import collections
import csv
import sys

rows = []
pre = sys.argv[2] if len(sys.argv) > 2 else "k_wf_"
for d in csv.DictReader(open(sys.argv[1])):
    name = d["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
    if name.startswith(pre) and not name.endswith("true>") and ", true>" not in name[-8:]:
        rows.append((int(d["Start_Timestamp"]), int(d["End_Timestamp"]), name, d.get("Stream_Id", d.get("Queue_Id", "0"))))
rows.sort()
# group per stream; a batch part starts at each k_wf_generate (or the first GEN step)
per_stream = collections.defaultdict(list)
for r in rows:
    per_stream[r[3]].append(r)
acc = collections.defaultdict(list)
for st, rs in per_stream.items():
    idx = 0
    for a, b, name, _ in rs:
        if name.startswith("k_wf_generate") or name.startswith("k_wf_accum"):
            idx = 0
            continue
        acc[(idx, name.split("<")[0])].append((b - a) / 1e3)
        idx += 1
tot = sum(sum(v) for v in acc.values())
for (i, n), v in sorted(acc.items()):
    print(f"launch {i:2d} {n:22s} n={len(v):4d} mean {sum(v)/len(v):8.1f} us  share {100*sum(v)/tot:5.1f} %")

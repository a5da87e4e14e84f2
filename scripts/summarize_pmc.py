#!/usr/bin/env python3
"""Per-kernel summary of a gpu_profile.sh output directory: kernel-trace stats (calls, avg us,
share of GPU time) and every PMC counter averaged per dispatch, plus derived ratios
(lane utilisation = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU), SALU/VALU, wait share).

usage: summarize_pmc.py gpurun_out/<tag> [kernel-substring ...]
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    for pre in ("void pt::", "pt::"):
        if name.startswith(pre):
            name = name[len(pre):]
    return name[:60]


def main():
    d = sys.argv[1]
    pick = sys.argv[2:]
    stats = {}
    ks = glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))
    if ks:
        with open(ks[0]) as f:
            for row in csv.DictReader(f):
                stats[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3, float(row["Percentage"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per[(short(row["Kernel_Name"]), row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        for (k, _), cs in per.items():
            for n, v in cs.items():
                ctr[k][n].append(v)
    names = sorted(set(stats) | set(ctr), key=lambda k: -stats.get(k, (0, 0, 0))[2])
    for k in names:
        if pick and not any(p in k for p in pick):
            continue
        calls, avg, pct = stats.get(k, (0, 0.0, 0.0))
        print(f"== {k}: calls {calls} avg {avg:.1f} us  {pct:.1f}% of GPU time")
        m = {n: sum(v) / len(v) for n, v in ctr[k].items()}
        for n in sorted(m):
            print(f"   {n:24s} {m[n]:.4g}")
        if m.get("SQ_ACTIVE_INST_VALU"):
            print(f"   lane_util                {m.get('SQ_THREAD_CYCLES_VALU', 0) / (64 * m['SQ_ACTIVE_INST_VALU']):.3f}")
        if m.get("SQ_INSTS_VALU"):
            print(f"   salu/valu                {m.get('SQ_INSTS_SALU', 0) / m['SQ_INSTS_VALU']:.3f}")
        if m.get("SQ_WAVE_CYCLES"):
            print(f"   wait_any/wave_cycles     {m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES']:.3f}")
            print(f"   wait_inst/wave_cycles    {m.get('SQ_WAIT_INST_ANY', 0) / m['SQ_WAVE_CYCLES']:.3f}")


if __name__ == "__main__":
    main()

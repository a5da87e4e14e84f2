#!/usr/bin/env python3
"""Busy time of the render kernel from a rocprofv3 --kernel-trace of bench.py (verdict r02 item 2):
the union of the dispatch intervals [Start_Timestamp, End_Timestamp] of the timed instances of the
dominant kernel, per step — the rocprof counterpart of bench.py's HIP-event `kernel_busy_ms_per_step`
(the batch's two parts run on their own streams, so their launches overlap: the summed per-dispatch
durations over-count the kernel's wall time, the union does not).

usage: trace_union.py KERNEL_TRACE_CSV BENCH_LINE_JSON [out.json]
out.json is keyed by the workload (WxHxsppxdepthxworld, as profiles/traffic.json); bench.py reports
the entry matching its configuration next to its own event union.
The bench line gives the kernel, launches per step and steps; the timed steps are the last
steps x launches_per_step dispatches of the kernel's uncounted instances (COUNT = false: the counted
render before the warm-up uses the COUNT = true instances)."""
import csv
import json
import sys

PREFIX = {"k_wf_step": ("k_wf_step_bf<",), "k_wf_trace": ("k_wf_trace<", "k_wf_trace_bf<")}


def uncounted(name: str, kernel: str) -> bool:
    args = [a.strip() for a in name[name.find("<") + 1:name.rfind(">")].split(",")]
    if name.startswith("k_wf_step_bf<"):  # <EXT, LDS, rcp, COUNT, GEN>
        return len(args) >= 4 and args[3] == "false"
    if name.startswith("k_wf_trace<"):  # <LDS, TRAV, COUNT, RING, PRUN>
        return len(args) >= 3 and args[2] == "false"
    return bool(args) and args[-1] == "false"


def union_ms(iv):
    iv = sorted(iv)
    busy, lo, hi = 0, None, None
    for a, b in iv:
        if hi is None or a > hi:
            if hi is not None:
                busy += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    if hi is not None:
        busy += hi - lo
    return busy / 1e6  # ns -> ms


def main():
    trace, line_path = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    line = [json.loads(x) for x in open(line_path) if x.startswith("{")][0]
    r = line["roofline"]
    kernel, per_step, steps = r["kernel"], int(round(r["launches_per_step"])), line["steps"]
    rows = []
    for d in csv.DictReader(open(trace)):
        name = d["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
        if name.startswith(PREFIX.get(kernel, (kernel + "<",))) and uncounted(name, kernel):
            rows.append((int(d["Start_Timestamp"]), int(d["End_Timestamp"]), name))
    rows.sort()
    timed = rows[-steps * per_step:]
    steps_ms = [union_ms([(a, b) for a, b, _ in timed[k * per_step:(k + 1) * per_step]]) for k in range(steps)]
    busy = sum(steps_ms) / steps
    durations = [(b - a) / 1e6 for a, b, _ in timed]
    res = {"kernel": kernel, "dispatches_timed": len(timed), "launches_per_step": per_step, "steps": steps,
           "busy_ms_per_step_rocprof": round(busy, 3), "busy_ms_steps_rocprof": [round(x, 3) for x in steps_ms],
           "sum_dispatch_ms_per_step_rocprof": round(sum(durations) / steps, 3),
           "avg_dispatch_ms_rocprof": round(sum(durations) / max(1, len(durations)), 4),
           "busy_ms_per_step_hip_events": r["kernel_busy_ms_per_step"],
           "avg_dispatch_ms_hip_events": r["kernel_avg_ms"],
           "busy_ratio_rocprof_over_events": round(busy / r["kernel_busy_ms_per_step"], 4),
           "bytes_per_launch": r["bytes_per_launch"],
           "achieved_gbs_rocprof": round(r["bytes_per_launch"] * per_step / (busy * 1e-3) / 1e9, 2),
           "workload": line["config"]["workload"], "source": trace}
    if out:
        import os
        import re
        m = re.search(r"(\d+)x(\d+) (\d+)spp depth (\d+)", line["config"]["workload"])
        key = f"{m.group(1)}x{m.group(2)}x{m.group(3)}x{m.group(4)}x{line['n_gpus']}"
        t = json.load(open(out)) if os.path.exists(out) else {}
        t[key] = res
        json.dump(t, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

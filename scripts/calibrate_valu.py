#!/usr/bin/env python3
"""VALU issue calibration (verdict r02 item 2).  Two modes:

  calibrate_valu.py run [--iters N --reps R]
      runs pt_selftest_valu (8 independent v_fma_f32 chains per thread, 8 waves per SIMD: VALU
      issue at the SIMD's peak) and prints its event time, its v_fma_f32 wave-instructions and the
      achieved f32 rate; under `rocprofv3 --pmc ...` this is the PMC pass of the calibration.
  calibrate_valu.py summarize DIR RUN_LOG [out.json]
      reads the rocprofv3 counter CSVs under DIR (the pass above) and the printed run line, and
      derives the constant of the issue formula: a kernel that issues one v_fma_f32 wave-instruction
      every `c` SIMD cycles (its measured peak) must read 1.0.  With SIMD-cycles = 128 x
      GRBM_GUI_ACTIVE (GRBM summed over 8 XCDs of 32 CUs x 4 SIMDs),
          valu_issue = k x SQ_ACTIVE_INST_VALU / (128 x GRBM_GUI_ACTIVE)
      and k is chosen so the microkernel reads 1.0; the same for SQ_INSTS_VALU.  Written to
      profiles/valu_calibration.json, which scripts/summarize_traffic.py applies.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brown-cs2240-path-tracer_amd"))


def run(argv):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--packed", action="store_true", help="v_pk_fma_f32 chains (two FMAs per lane each)")
    ap.add_argument("--mixed", action="store_true", help="packed and plain chains interleaved (1 : 2)")
    ap.add_argument("--dep", choices=["packed", "plain"], help="two dependent chains per thread")
    a = ap.parse_args(argv)
    import pt_amd
    mode = 2 if a.mixed else (3 if a.dep == "packed" else 4) if a.dep else int(a.packed)
    ms, n = pt_amd.selftest_valu(a.iters, a.reps, mode)
    cus = 256
    # achieved rate: 2 flops per lane per FMA (x2 packed), 64 lanes per wave-instruction
    flops_per_instr = 4 / 3 if a.mixed else 2 if (a.packed or a.dep == "packed") else 1
    tflops = n * 64 * 2 * flops_per_instr / (ms * 1e-3) / 1e12
    name = "k_selftest_valu" + ("_mix" if a.mixed else ("_dep_" + a.dep) if a.dep else "_pk" if a.packed else "")
    print(json.dumps({"kernel": name, "iters": a.iters, "reps": a.reps, "ms": ms,
                      "fma_wave_instr": n, "fma_wave_instr_per_launch": n // a.reps, "tflops_f32": round(tflops, 2),
                      "wave_instr_per_simd_per_ns": n / (cus * 4) / (ms * 1e6)}), flush=True)


def summarize(d, log, out):
    agg = collections.defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_selftest_valu" not in r["Kernel_Name"]:
                continue
            c = agg[r["Dispatch_Id"]]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not agg:
        raise SystemExit("no k_selftest_valu dispatch in " + d)
    line = [json.loads(x) for x in open(log) if x.startswith("{")][0]
    per = line["fma_wave_instr_per_launch"]
    disp = sorted(agg.items(), key=lambda kv: int(kv[0]))
    last = disp[-1][1]  # the warm launch's clock ramp is over by the last dispatch
    simd_cycles = 128.0 * last["GRBM_GUI_ACTIVE"]
    ks = sorted(128.0 * c["GRBM_GUI_ACTIVE"] / c["SQ_ACTIVE_INST_VALU"] for _, c in disp[1:] if c.get("SQ_ACTIVE_INST_VALU"))
    res = {"_source": "scripts/calibrate_valu.sh: rocprofv3 --pmc of scripts/calibrate_valu.py run (pt_selftest_valu: "
                      "8 independent v_fma_f32 chains per thread, 32 FMAs per loop iteration, 8 waves per SIMD)",
           "dispatches": len(disp), "counters_last_dispatch": last, "fma_wave_instr_per_launch": per,
           "run_line": line}
    res["insts_valu_per_fma"] = last.get("SQ_INSTS_VALU", 0.0) / per  # counter coverage vs the known count
    if last.get("SQ_ACTIVE_INST_VALU"):
        # k such that k * ACTIVE / SIMD-cycles = 1 for this peak-issue kernel
        res["k_active"] = simd_cycles / last["SQ_ACTIVE_INST_VALU"]
    if last.get("SQ_INSTS_VALU"):
        res["k_insts"] = simd_cycles / last["SQ_INSTS_VALU"]
    # cycles per v_fma_f32 wave-instruction at peak, from the counters' own clock
    res["simd_cycles_per_fma"] = simd_cycles / per
    res["old_formula_reads"] = 4.0 * last.get("SQ_ACTIVE_INST_VALU", 0.0) / simd_cycles
    if ks:  # spread over the timed dispatches (the first is the warm-up launch)
        res["k_active_dispatches"] = {"min": ks[0], "median": ks[len(ks) // 2], "max": ks[-1], "n": len(ks)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "summarize":
        summarize(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else "profiles/valu_calibration.json")
    else:
        run(sys.argv[2:] if len(sys.argv) > 1 and sys.argv[1] == "run" else sys.argv[1:])

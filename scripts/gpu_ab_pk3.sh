#!/bin/bash
# in-process A/B: default vs phase 1 two packed pairs at a time (ablib/pk3, extension instances)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
timeout -k 10 300 python3 scripts/ab_libs.py $B ablib/pk3/libpt_hip.so --async-torch --rounds 7 > gpurun_out/ab_pk3a.log 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_libs.py ablib/pk3/libpt_hip.so $B --async-torch --rounds 7 > gpurun_out/ab_pk3b.log 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_pk3*.log
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcpk_pk3 -o run -- python3 scripts/render_lib.py ablib/pk3/libpt_hip.so --spp 16 --reps 1 > gpurun_out/pmcpk_pk3.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections, json
agg = collections.defaultdict(lambda: collections.defaultdict(float)); ids = collections.defaultdict(set)
for d in csv.DictReader(open("gpurun_out/pmcpk_pk3/run_counter_collection.csv")):
    name = d["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
    if not name.startswith("k_wf_step_bf<"): continue
    agg[name][d["Counter_Name"]] += float(d["Counter_Value"]); ids[name].add(d["Dispatch_Id"])
for name, c in sorted(agg.items()):
    print("pk3", name, len(ids[name]), json.dumps({k: round(x / len(ids[name])) for k, x in sorted(c.items())}))
PY

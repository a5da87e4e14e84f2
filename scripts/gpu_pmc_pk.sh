#!/bin/bash
# PMC of the fused kernel's extension instance: default build vs phase 1 in packed pairs (ablib/pk)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY"
for V in base pk; do
  LIB=brown-cs2240-path-tracer_amd/lib/libpt_hip.so; [ $V = pk ] && LIB=ablib/pk/libpt_hip.so
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcpk_$V -o run -- python3 scripts/render_lib.py $LIB --spp 16 --reps 1 > gpurun_out/pmcpk_$V.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, collections, json
for v in ("base", "pk"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for d in csv.DictReader(open(f"gpurun_out/pmcpk_{v}/run_counter_collection.csv")):
        name = d["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
        if not name.startswith("k_wf_step_bf<"): continue
        agg[name][d["Counter_Name"]] += float(d["Counter_Value"])
        n[(name, d["Dispatch_Id"])] += 0
    for name, c in sorted(agg.items()):
        disp = len({k for k in n if k[0] == name})
        print(v, name, "dispatches", disp, json.dumps({k: round(x / disp) for k, x in sorted(c.items())}))
PY

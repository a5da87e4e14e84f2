#!/bin/bash
# PMC of the injection builds: SQ_INSTS_VALU / SQ_INSTS_SALU / GRBM_GUI_ACTIVE of the
# bench's k_wf_step_bf dispatches (64 spp) for the default build and ablib/pad16, so the injected
# instructions are counted, not estimated -> gpurun_out/pmc_pad/summary.json
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
O=gpurun_out/pmc_pad
rm -rf $O; mkdir -p $O
cp $L $O/base.so
for v in base pad16 salu16; do
  if [ $v = base ]; then cp $O/base.so $L; else cp ablib/$v/libpt_hip.so $L; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/$v -o run \
    -- python3 bench.py --steps 1 --warmup 0 --spp 64 --no-cpu-baseline > $O/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; if [ $rc -ne 0 ]; then cp $O/base.so $L; exit $rc; fi
done
cp $O/base.so $L
python3 - <<'PY'
import collections, csv, glob, json
out = {}
for v in ("base", "pad16", "salu16"):
    agg = collections.defaultdict(float)
    disp = set()
    for f in glob.glob(f"gpurun_out/pmc_pad/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_wf_step_bf" not in k:
                continue
            args = k.split("<")[1].split(">")[0].split(",")
            if args[3].strip() != "false":  # COUNT instances: the bench's untimed counted render
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    out[v] = dict(agg, dispatches=len(disp))
json.dump(out, open("gpurun_out/pmc_pad/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY

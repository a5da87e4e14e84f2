cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02f_kt -o run -- python3 scripts/env_ab.py --reps 1 PT_REGEN=0,PT_PARTS=1 PT_REGEN=1,PT_PARTS=1 > gpurun_out/r02f_kt.log 2>&1; rc=$?
grep -h '^{' gpurun_out/r02f_kt.log; python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r02f_kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wf_" in r["Name"]:
            print(r["Name"].split("(")[0][:90], r["Calls"], round(float(r["AverageNs"])/1e3,1), "us avg", round(float(r["TotalDurationNs"])/1e6,2), "ms total")
PY
exit $rc

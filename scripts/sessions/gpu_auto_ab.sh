cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for cfg in "CornellBox 128 1" "CornellBox 256 1" "CornellBox 512 1" "CornellBox-Glossy 128 1" "CornellBox-Glossy 256 1" "CornellBox-Glossy 512 1" "MedievalBoat 256 1"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/env_ab.py --scene $1 --width $2 --height $2 --depth 16 --spp $3 --reps 3 PT_KERNEL=mega PT_KERNEL=wavefront > gpurun_out/autoab.log 2>&1 || exit 1
  echo "$cfg $(grep '^{' gpurun_out/autoab.log | python3 -c 'import sys,json; print([json.loads(l)["ms"] for l in sys.stdin])')"
done

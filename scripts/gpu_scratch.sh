cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 2 --depth 16 --reps 1 PT_PIPE=0 > gpurun_out/r02n.log 2>&1; tail -5 gpurun_out/r02n.log | cut -c1-300
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u scripts/env_ab.py --scene MedievalBoat --width 512 --height 512 --spp 2 --depth 16 --reps 1 PT_PIPE=0 PT_PIPE=1 > gpurun_out/r02n2.log 2>&1; tail -5 gpurun_out/r02n2.log | cut -c1-300

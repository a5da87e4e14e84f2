cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/env_ab.py --scene MedievalBoat --width 1920 --height 1080 --spp 2 --depth 16 --reps 1 PT_BIG_LEAF=0 PT_BIG_LEAF=1000,PT_BIG_RATIO=64,PT_BIG_MODE=1 PT_BIG_LEAF=1000,PT_BIG_RATIO=1,PT_BIG_MODE=1 PT_BIG_LEAF=0,PT_PIPE=1 PT_BIG_LEAF=0,PT_TRAV=lean8 PT_BIG_LEAF=0,PT_TRAV=lean32 PT_BIG_LEAF=0,PT_NODE_BIAS=1 2>&1 | tee gpurun_out/r02j_ab.log

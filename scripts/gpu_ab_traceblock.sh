#!/bin/bash
# In-process A/B of k_wf_trace's block size (make EXTRA=-DPT_TRACE_BLOCK=n OUT_DIR=../../ablib/tbN):
# LDS per block = max_stack x block x 4 (lane stacks) + waves x kStageBytes, so smaller blocks pack the
# CU's 160 KB more finely -> gpurun_out/ab_tb_*.log
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
for sc in "CornellBox-Glossy --depth 16 --spp 32" "MedievalBoat --res 512 --depth 16 --spp 16"; do
  n=$(echo $sc | cut -d' ' -f1)
  timeout -k 10 400 python3 scripts/ab_libs.py $B ablib/tb256/libpt_hip.so ablib/tb128/libpt_hip.so --async-torch --rounds 3 --scene $sc > gpurun_out/ab_tb_${n}_1.log 2>&1 || exit $?
  timeout -k 10 400 python3 scripts/ab_libs.py ablib/tb128/libpt_hip.so ablib/tb256/libpt_hip.so $B --async-torch --rounds 3 --scene $sc > gpurun_out/ab_tb_${n}_2.log 2>&1 || exit $?
done
grep -h '^{' gpurun_out/ab_tb_*.log

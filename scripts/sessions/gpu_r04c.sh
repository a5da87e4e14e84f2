#!/bin/bash
# Round 4: parity suite on the current build, the exhaustive div_r check, in-process A/B of the
# replay's skipped leaf boxes + div_r against the previous build, then scripts/gpu_r04b.sh.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/profiles/r04c_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/profiles/r04c_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/check_div.py > gpurun_out/profiles/r04c_check_div.log 2>&1
rc=$?; echo "check_div rc=$rc"; tail -1 gpurun_out/profiles/r04c_check_div.log; if [ $rc -gt 1 ]; then exit $rc; fi
L=brown-cs2240-path-tracer_amd/lib/libpt_hip.so
AB=gpurun_out/profiles/r04c_ab_replay_div.log
: > $AB
for sc in CornellBox CornellBox-Mirror; do
  for order in "$L ablib/base/libpt_hip.so ablib/skip/libpt_hip.so ablib/div/libpt_hip.so ablib/rcp/libpt_hip.so" "ablib/rcp/libpt_hip.so ablib/div/libpt_hip.so ablib/skip/libpt_hip.so ablib/base/libpt_hip.so $L"; do
    d=8; [ $sc = CornellBox-Mirror ] && d=16
    echo "== $sc depth $d order: $order" >> $AB
    timeout -k 10 300 python3 scripts/ab_libs.py $order --scene $sc --res 1024 --spp 64 --depth $d --rounds 5 --async-torch >> $AB 2>&1
    rc=$?; echo "ab $sc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
# a rank's share at N = 8 (32 frames: one batch, its tails weigh twice) — the early exit of idle blocks
for order in "$L ablib/rcp/libpt_hip.so ablib/base/libpt_hip.so" "ablib/base/libpt_hip.so ablib/rcp/libpt_hip.so $L"; do
  echo "== CornellBox depth 8, 32 frames, order: $order" >> $AB
  timeout -k 10 300 python3 scripts/ab_libs.py $order --scene CornellBox --res 1024 --spp 32 --depth 8 --rounds 7 --async-torch >> $AB 2>&1
  rc=$?; echo "ab share rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -v "^ *$" $AB | tail -40
bash scripts/gpu_r04b.sh
# the box's own toolchain builds HEAD: the sources of the shipped library, built from scratch in a
# scratch directory, give a library whose build id is the shipped one's
rm -rf /tmp/boxbuild && mkdir -p /tmp/boxbuild && cp -r brown-cs2240-path-tracer_amd include /tmp/boxbuild/ && rm -rf /tmp/boxbuild/brown-cs2240-path-tracer_amd/lib
( cd /tmp/boxbuild/brown-cs2240-path-tracer_amd/csrc && time timeout -k 10 600 make -s -j16 ) > gpurun_out/profiles/r04c_box_build.log 2>&1
rc=$?; echo "box build rc=$rc" | tee -a gpurun_out/profiles/r04c_box_build.log
python3 - >> gpurun_out/profiles/r04c_box_build.log 2>&1 <<'PY'
import ctypes
ids = []
for p in ("brown-cs2240-path-tracer_amd/lib/libpt_hip.so", "/tmp/boxbuild/brown-cs2240-path-tracer_amd/lib/libpt_hip.so"):
    L = ctypes.CDLL(p); L.pt_build_id.restype = ctypes.c_char_p; ids.append(L.pt_build_id().decode()); print(p, ids[-1])
print("same build id:", ids[0] == ids[1])
PY
tail -3 gpurun_out/profiles/r04c_box_build.log

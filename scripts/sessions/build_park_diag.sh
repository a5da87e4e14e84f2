#!/bin/bash
# Diagnostic build (verdict r03 item 3, step 3): how many lanes of a wave are parked at the SAME
# big leaf when a cooperative turn starts.  A copy of the sources with three counter increments in
# the counting instances of trav_step_lean (pt_device.h), built to ablib/parkdiag; the product
# sources are untouched.  Per turn, lane f (the lane served) adds 1 to box_tests, the number of
# parked lanes to shadow_queries and the number parked at f's leaf to nodes — counted renders of
# this build minus those of the product build (whose counters are the reference's work, the same
# in both) give turns, parked lanes and same-leaf lanes (scripts/ab_libs.py --counters).
set -eu
cd "$(dirname "$0")/.."
T=/tmp/parkdiag
rm -rf $T && mkdir -p $T && cp -r brown-cs2240-path-tracer_amd include $T/
python3 - $T/brown-cs2240-path-tracer_amd/csrc/pt_device.h <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """            int my0 = 0, myn = 0;  // the first parked lane's leaf (the other lanes' fields may not be a leaf's)
            big_seg(s, my0, myn);
"""
assert old in s
new = old + """            if constexpr (COUNT) {
                const int f_ = (int)__builtin_ctzll(parked);
                const int r0_ = __builtin_amdgcn_readlane(my0, f_);
                const uint64_t same_ = __ballot(((state & TF_PARK) != 0) && my0 == r0_);
                if ((int)(threadIdx.x & 63u) == f_) {
                    cnt.box_tests += 1;
                    cnt.shadow_queries += (uint64_t)__popcll(parked);
                    cnt.nodes += (uint64_t)__popcll(same_);
                }
            }
"""
open(p, "w").write(s.replace(old, new))
PY
make -s -j8 -C $T/brown-cs2240-path-tracer_amd/csrc OUT_DIR=$PWD/ablib/parkdiag $PWD/ablib/parkdiag/libpt_hip.so
ls -la ablib/parkdiag/libpt_hip.so

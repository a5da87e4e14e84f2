#!/usr/bin/env python3
"""Exhaustive device check of the division-free reciprocal (pt_math.h rcp_rn) vs IEEE 1/x."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "brown-cs2240-path-tracer_amd"))
import pt_amd  # noqa: E402

RANGES = {
    "normal 2^-126..2^125": (0x00800000, 0x7E000000),
    "large 2^125..inf": (0x7E000000, 0x7F800000),
    "subnormal x": (0x00000001, 0x007FFFFF),
}
for steps in (0, 1, 2):
    for name, (lo, hi) in RANGES.items():
        t = time.time()
        m, b = pt_amd.selftest_rcp(steps, lo, hi)
        print(f"steps={steps} {name}: mismatches={m} example=0x{b:08x} ({time.time() - t:.3f}s)", flush=True)

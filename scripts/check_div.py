#!/usr/bin/env python3
"""Exhaustive check of pt_math.h div_r on the device: every pair of f32 mantissas (a, b in [1, 2),
2^46 pairs) — the case every in-range quotient scales to — plus 2^34 random bit
patterns of any exponent.  Prints one progress line per slice; exit status 1 on any mismatch.
usage: check_div.py [--slices 64]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brown-cs2240-path-tracer_amd"))
import pt_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", type=int, default=64)
    a = ap.parse_args()
    n = 1 << 23
    step = n // a.slices
    total, bad = 0, 0
    t0 = time.time()
    for k in range(a.slices):
        m, fa, fb = pt_amd.selftest_div(0, 0, n, k * step, step)
        total += n * step
        bad += m
        print(f"slice {k + 1}/{a.slices}: a mantissas [{k * step}, {(k + 1) * step}) x all b: {m} mismatches"
              + (f" (e.g. a={fa:#010x} b={fb:#010x})" if m else "") + f", {time.time() - t0:.1f} s", flush=True)
    for s in range(16):
        m, fa, fb = pt_amd.selftest_div(1, 0, 1 << 22, 0, 256, seed=1000 + s)
        total += (1 << 22) * 256
        bad += m
        print(f"random {s + 1}/16: {1 << 30} pairs of any bits: {m} mismatches", flush=True)
    print(f"pairs checked {total}, mismatches {bad}, {time.time() - t0:.1f} s")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())

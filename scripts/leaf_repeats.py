#!/usr/bin/env python3
"""How often does a ray of the reference's traversal test an entry it has already tested?  A host
model of intersect() (src/wgsl-util/intersection-logic.wgsl:1-215: right-then-left stack walk,
exit-distance pruning, leaf children tested in order) over a packed scene (pt-pack.js output dir),
in float64 (counts, not bits), for camera-like rays from `eye` into the scene box and two bounce
rays from each hit.  Prints the tree's leaf statistics, tests per ray, distinct entries per ray,
and how many repeats a per-ray direct-mapped table of S slots (uid mod S) would catch.
usage: leaf_repeats.py PACKED_DIR [eye x,y,z] [rays]"""
import collections
import sys

import numpy as np


def main():
    d = sys.argv[1]
    b = np.fromfile(d + "/bvh_data.f32", np.float32).astype(np.float64)
    t = np.fromfile(d + "/triangle_data.f32", np.float32).astype(np.float64)
    V = t[int(t[2]):int(t[2]) + int(t[0]) * 3].reshape(-1, 3)
    leaves = {}

    def walk(i):
        if b[i] == 1:
            e = b[i + 17:i + 17 + int(b[i + 4])].reshape(-1, 4).astype(int)
            leaves[i] = [tuple(x[:3]) for x in e]
            return
        walk(int(b[i + 2]))
        walk(int(b[i + 3]))
    walk(6)
    uid = {}
    for i in sorted(leaves):
        for k in leaves[i]:
            uid.setdefault(k, len(uid))
    E = sum(len(v) for v in leaves.values())
    print(f"leaves {len(leaves)} entries {E} distinct {len(uid)} max leaf {max(map(len, leaves.values()))}")

    def box(o, inv, mn, mx):
        t1, t2 = (mn - o) * inv, (mx - o) * inv
        tmin, tmax = max(-3e38, np.max(np.minimum(t1, t2))), min(3e38, np.min(np.maximum(t1, t2)))
        return (tmin if tmin > 0 else tmax) if tmax > max(tmin, 0) else -1.0

    def tri(o, dd, k):
        v0, v1, v2 = V[k[0] - 1], V[k[1] - 1], V[k[2] - 1]
        e1, e2 = v1 - v0, v2 - v0
        h = np.cross(dd, e2)
        a = e1 @ h
        if -1e-8 < a < 1e-8:
            return None
        f = 1 / a
        s = o - v0
        u = f * (s @ h)
        if u < 0 or u > 1:
            return None
        q = np.cross(s, e1)
        v = f * (dd @ q)
        if v < 0 or u + v > 1:
            return None
        tt = f * (e2 @ q)
        return tt if tt > 1e-8 else None

    SL = (8, 16, 32, 64)
    caught = dict.fromkeys(SL, 0)

    def intersect(o, dd):
        with np.errstate(divide="ignore"):
            inv = 1 / dd
        stack, sp, ct, tests, seen, best = [6], 0, -1.0, 0, set(), None
        tabs = {S: [-1] * S for S in SL}
        while sp > -1:
            p = stack[sp]
            ld, rd = box(o, inv, b[p + 5:p + 8], b[p + 8:p + 11]), box(o, inv, b[p + 11:p + 14], b[p + 14:p + 17])
            li, ri, ll, rl = 0 < ld, 0 < rd, False, False
            for side, hit in ((2, li), (3, ri)):
                c = int(b[p + side])
                if not hit or b[c] != 1:
                    continue
                ll, rl = (True, rl) if side == 2 else (ll, True)
                for k in leaves[c]:
                    tests += 1
                    u = uid[k]
                    for S, tb in tabs.items():
                        caught[S] += tb[u % S] == u
                        tb[u % S] = u
                    seen.add(k)
                    tt = tri(o, dd, k)
                    if tt is not None and (ct < 0 or tt < ct):
                        ct, best = tt, k
            tl = li and not ll and not (ct > 0 and ld > ct)
            tr = ri and not rl and not (ct > 0 and rd > ct)
            if not tl and not tr:
                sp -= 1
                while sp >= 0 and stack[sp] == -1:
                    sp -= 1
            else:
                stack += [0] * (sp + 3 - len(stack))
                stack[sp] = -1
                if tl and not tr:
                    sp += 1
                    stack[sp] = int(b[p + 2])
                elif tr and not tl:
                    sp += 1
                    stack[sp] = int(b[p + 3])
                else:
                    stack[sp + 1] = int(b[p + 2])
                    sp += 2
                    stack[sp] = int(b[p + 3])
        return ct, best, tests, len(seen)

    rng = np.random.default_rng(1)
    eye = np.array([float(x) for x in sys.argv[2].split(",")]) if len(sys.argv) > 2 else np.array([0.0, 1.0, 3.5])
    nr = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    lo, hi = b[0:3], b[3:6]
    T = D = n = 0
    for _ in range(nr):
        dd = lo + (hi - lo) * rng.random(3) - eye
        dd /= np.linalg.norm(dd)
        ct, best, tests, dist = intersect(eye, dd)
        T, D, n = T + tests, D + dist, n + 1
        if best is not None:
            p = eye + ct * dd
            for _ in range(2):
                d2 = rng.normal(size=3)
                d2 /= np.linalg.norm(d2)
                _, _, t2, di2 = intersect(p + 1e-4 * d2, d2)
                T, D, n = T + t2, D + di2, n + 1
    print(f"rays {n}: tests per ray {T / n:.1f}, distinct entries per ray {D / n:.1f}, repeats {1 - D / T:.3f}")
    print("repeats caught per ray by a direct-mapped per-ray table of S slots: " +
          ", ".join(f"S={S}: {v / n:.1f}" for S, v in caught.items()))


if __name__ == "__main__":
    main()

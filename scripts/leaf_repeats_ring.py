#!/usr/bin/env python3
"""Which of a ray's repeated leaf-entry tests could an exact skip catch, and with what state?
A host model of intersect() (src/wgsl-util/intersection-logic.wgsl:1-215; the same walk as
leaf_repeats.py, float64: counts, not bits) over a packed scene (pt-pack.js output dir).  Per ray it
records the leaves it tests in order and classifies every repeated test (an entry whose (i0, i1, i2,
material) the ray tested before):
  pair   — the entry is also in the left leaf of the same pair (both leaf children hit): a static fact
           of the node, needs no per-ray state;
  ringK  — the entry is in one of the ray's last K tested leaves (the pair's left leaf included);
  any    — every repeat (the ray's full tested set).
usage: leaf_repeats_ring.py PACKED_DIR [eye x,y,z] [rays]"""
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
            leaves[i] = [tuple(x) for x in e]
            return
        walk(int(b[i + 2]))
        walk(int(b[i + 3]))
    walk(6)
    uid = {}
    for i in sorted(leaves):
        for k in leaves[i]:
            uid.setdefault(k, len(uid))
    lset = {i: {uid[k] for k in v} for i, v in leaves.items()}
    E = sum(len(v) for v in leaves.values())
    print(f"leaves {len(leaves)} entries {E} distinct {len(uid)} max leaf {max(map(len, leaves.values()))}")
    # static: for every internal node with two leaf children, right entries also in the left leaf
    npairs = nd = 0
    def walk2(i):
        nonlocal npairs, nd
        if b[i] == 1:
            return
        l, r = int(b[i + 2]), int(b[i + 3])
        if b[l] == 1 and b[r] == 1:
            npairs += 1
            nd += len(lset[l] & lset[r])
        walk2(l); walk2(r)
    walk2(6)
    # the fixed visit order of leaves: at a node its leaf children (left, right), then its internal
    # children, right subtree first (intersection-logic.wgsl: right pushed on top)
    order = []
    def walk3(i):
        l, r = int(b[i + 2]), int(b[i + 3])
        if b[l] == 1: order.append(l)
        if b[r] == 1: order.append(r)
        if b[r] != 1: walk3(r)
        if b[l] != 1: walk3(l)
    walk3(6)
    spred = {order[i]: (order[i - 1] if i else None) for i in range(len(order))}
    # static alternatives per leaf: the A nearest predecessors in the visit order that share
    # entries with it; or the A leaves (earlier in the order) sharing the most entries with it
    opos = {c: i for i, c in enumerate(order)}
    AS = (1, 2, 4, 8)
    near = {c: [m for m in reversed(order[:opos[c]]) if lset[m] & lset[c]] for c in order}
    most = {c: sorted(order[:opos[c]], key=lambda m: -len(lset[m] & lset[c])) for c in order}
    print(f"nodes with two leaf children {npairs}, right entries also in the left leaf {nd}")

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

    KS = (1, 2, 4, 8, 16)
    tot = {"tests": 0, "any": 0, "pair": 0, "static_pred": 0, **{f"near{A}": 0 for A in AS}, **{f"most{A}": 0 for A in AS}, **{f"ring{K}": 0 for K in KS}}
    pairfreq = {}  # (leaf, last) -> repeats caught by skipping last's entries

    def intersect(o, dd):
        with np.errstate(divide="ignore"):
            inv = 1 / dd
        stack, sp, ct, best = [6], 0, -1.0, None
        seen, visited = set(), []
        while sp > -1:
            p = stack[sp]
            ld, rd = box(o, inv, b[p + 5:p + 8], b[p + 8:p + 11]), box(o, inv, b[p + 11:p + 14], b[p + 14:p + 17])
            li, ri, ll, rl = 0 < ld, 0 < rd, False, False
            pair_left = None
            for side, hit in ((2, li), (3, ri)):
                c = int(b[p + side])
                if not hit or b[c] != 1:
                    continue
                ll, rl = (True, rl) if side == 2 else (ll, True)
                last = visited[-1] if visited else None
                for k in leaves[c]:
                    u = uid[k]
                    if last is not None and last == spred[c] and u in lset[last]:
                        tot["static_pred"] += 1
                    if last is not None and u in lset[last]:
                        pairfreq[(c, last)] = pairfreq.get((c, last), 0) + 1
                        if f"probe1" in tot:
                            for A in AS:
                                tot[f"probe{A}"] += last in pchoice.get(c, [])[:A]
                                tot[f"hyb{A}"] += last in hchoice[c][:A]
                        for A in AS:
                            tot[f"near{A}"] += last in near[c][:A]
                            tot[f"most{A}"] += last in most[c][:A]
                    tot["tests"] += 1
                    if u in seen:
                        tot["any"] += 1
                        if side == 3 and pair_left is not None and u in lset[pair_left]:
                            tot["pair"] += 1
                        for K in KS:
                            if any(u in lset[m] for m in visited[-K:]):
                                tot[f"ring{K}"] += 1
                    seen.add(u)
                    tt = tri(o, dd, k)
                    if tt is not None and (ct < 0 or tt < ct):
                        ct, best = tt, k
                visited.append(c)
                if side == 2:
                    pair_left = c
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
        return ct, best

    # probe: rays leaving random points of random triangles in uniform directions (no camera)
    prng = np.random.default_rng(7)
    np_ = int(sys.argv[4]) if len(sys.argv) > 4 else 600
    allk = [k for v in leaves.values() for k in v]
    for _ in range(np_):
        k = allk[prng.integers(len(allk))]
        v0, v1, v2 = V[k[0] - 1], V[k[1] - 1], V[k[2] - 1]
        a, c = prng.random(2)
        if a + c > 1: a, c = 1 - a, 1 - c
        p = v0 + a * (v1 - v0) + c * (v2 - v0)
        d2 = prng.normal(size=3); d2 /= np.linalg.norm(d2)
        intersect(p + 1e-4 * d2, d2)
    probe = {}
    for (c, m), v in pairfreq.items():
        probe.setdefault(c, []).append((v, m))
    pchoice = {c: [m for _, m in sorted(v, reverse=True)] for c, v in probe.items()}
    hchoice = {}
    for c in order:  # probe's choices first, then the nearest sharing predecessors
        h = list(pchoice.get(c, []))
        h += [m for m in near[c] if m not in h]
        hchoice[c] = h
    pairfreq.clear()
    for key in list(tot): tot[key] = 0
    for A in AS: tot[f"probe{A}"] = 0; tot[f"hyb{A}"] = 0
    rng = np.random.default_rng(1)
    eye = np.array([float(x) for x in sys.argv[2].split(",")]) if len(sys.argv) > 2 else np.array([0.0, 1.0, 3.6])
    nr = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    lo, hi = b[0:3], b[3:6]
    n = 0
    for _ in range(nr):
        dd = lo + (hi - lo) * rng.random(3) - eye
        dd /= np.linalg.norm(dd)
        ct, best = intersect(eye, dd)
        n += 1
        if best is not None:
            p = eye + ct * dd
            for _ in range(2):
                d2 = rng.normal(size=3)
                d2 /= np.linalg.norm(d2)
                intersect(p + 1e-4 * d2, d2)
                n += 1
    byleaf = {}
    for (c, m), v in pairfreq.items():
        byleaf.setdefault(c, []).append(v)
    for A in AS:
        tot[f"freq{A}"] = sum(sum(sorted(v, reverse=True)[:A]) for v in byleaf.values())
    print(f"rays {n}: tests per ray {tot['tests'] / n:.1f}, repeats per ray {tot['any'] / n:.1f}")
    print("repeats caught per ray: " + ", ".join(f"{k} {v / n:.1f}" for k, v in tot.items() if k not in ("tests", "any")))


if __name__ == "__main__":
    main()

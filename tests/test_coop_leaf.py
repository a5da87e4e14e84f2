"""The cooperative big-leaf turn (pt_device.h big_turn) ends a leaf with the same closest hit as
the reference's sequential leaf loop (intersection-logic.wgsl test_leaf: entries in order, a hit
taken when t < the closest t so far, or when there is none yet), for any hit pattern, ties and
incoming closest t included: lane l keeps the first of its smallest-t hits among entries
l, l + 64, ..., a butterfly reduction over the 64 lanes keeps the smallest (t, entry), and the
ray's best changes only when that t is strictly smaller.  Host logic, no GPU."""
import random

import pytest

NONE = 0x7FFFFFFF


def sequential(ts, best_t, best):
    """ts[k]: t of entry k's hit, or None (no hit) — the reference's loop."""
    for k, t in enumerate(ts):
        if t is not None and (best_t < 0.0 or t < best_t):
            best_t, best = t, k
    return best_t, best


def cooperative(ts, best_t, best, lanes=64):
    bt = [0.0] * lanes
    bk = [NONE] * lanes
    for lane in range(lanes):
        for c in range(lane, len(ts), lanes):
            t = ts[c]
            if t is not None and (bk[lane] == NONE or t < bt[lane]):
                bt[lane], bk[lane] = t, c
    off = 1
    while off < lanes:  # __shfl_xor butterfly: every lane ends with the wave's minimum
        nt, nk = bt[:], bk[:]
        for lane in range(lanes):
            ot, ok = bt[lane ^ off], bk[lane ^ off]
            if ok != NONE and (bk[lane] == NONE or ot < bt[lane] or (ot == bt[lane] and ok < bk[lane])):
                nt[lane], nk[lane] = ot, ok
        bt, bk = nt, nk
        off <<= 1
    assert len(set(bk)) == 1 and len(set(bt)) == 1
    if bk[0] != NONE and (best_t < 0.0 or bt[0] < best_t):
        return bt[0], bk[0]
    return best_t, best


@pytest.mark.parametrize("seed", range(200))
def test_cooperative_leaf_matches_sequential(seed):
    rng = random.Random(seed)
    n = rng.choice([1, 5, 63, 64, 65, 128, 200, 777])
    levels = [rng.uniform(0.01, 10.0) for _ in range(rng.randint(1, 6))]  # few distinct t: many ties
    p_hit = rng.choice([0.0, 0.02, 0.3, 1.0])
    ts = [rng.choice(levels) if rng.random() < p_hit else None for _ in range(n)]
    best_t = rng.choice([-1.0, rng.choice(levels), rng.uniform(0.01, 10.0)])
    best = -1 if best_t < 0.0 else 10**6
    assert cooperative(ts, best_t, best) == sequential(ts, best_t, best)


def test_equal_t_keeps_the_earlier_leaf():
    ts = [None] * 100
    ts[70] = 2.0
    assert cooperative(ts, 2.0, 999) == (2.0, 999)  # strict <: the incoming best stays
    ts[3] = 2.0
    assert cooperative(ts, -1.0, -1) == (2.0, 3)  # first in leaf order among the smallest

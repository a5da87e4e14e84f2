"""The pooled leaf turn (pt_device.h lean_leaf_pool, round 4): a leaf lane's remaining entries
[k, lim) of its leaf pair are cut into runs of sc.leaf_pool positions (option pool_run: 2 or 4), the runs are tested by other
lanes in any order, each run keeps its smallest (t, position), the owner's key is the minimum of
the runs' (t, position) keys, and the result replaces the lane's closest hit only if strictly
closer.  Claim: that is exactly where the reference's leaf loop ends — entries in order, each hit
taken when `closest_t < 0 || t < closest_t` (src/wgsl-util/intersection-logic.wgsl:58-125) — ties
included (the first entry in pair order among equal t wins, and an equal t never displaces the
closest hit carried in from earlier pairs).  Host model with forced ties, no GPU."""
import random

import pytest

RUNS = (1, 2, 4, 8, 16)  # option pool_run takes 2 or 4; the claim holds for any run length


def reference_loop(ts, prior_t, prior_rec, k0):
    """ts[i]: t of entry i if it reports a hit, else None; entries k0.. in order."""
    best_t, best = prior_t, prior_rec
    for pos in range(k0, len(ts)):
        t = ts[pos]
        if t is not None and (best_t < 0 or t < best_t):
            best_t, best = t, pos
    return best_t, best


def pooled(ts, prior_t, prior_rec, k0, rng, run):
    runs = [(p, min(p + run, len(ts))) for p in range(k0, len(ts), run)]
    rng.shuffle(runs)  # any lane, any order
    key = None
    for p0, p1 in runs:
        bt, bk = float("inf"), None
        for pos in range(p0, p1):  # positions ascend: strict < keeps the first of equal t
            t = ts[pos]
            if t is not None and t < bt:
                bt, bk = t, pos
        if bk is not None and (key is None or (bt, bk) < key):
            key = (bt, bk)  # ds_min_u64 of (t bits << 32 | position): lexicographic (t, position)
    if key is not None and (prior_t < 0 or key[0] < prior_t):
        return key
    return prior_t, prior_rec


@pytest.mark.parametrize("run", RUNS)
@pytest.mark.parametrize("seed", range(40))
def test_pooled_turn_equals_the_reference_loop(seed, run):
    rng = random.Random(seed)
    for _ in range(200):
        n = rng.randint(1, 70)
        tvals = [0.25, 0.5, 0.5, 1.0, 1.0, 2.0, 3.5]  # few distinct values: ties everywhere
        ts = [rng.choice(tvals) if rng.random() < 0.4 else None for _ in range(n)]
        k0 = rng.randint(0, n - 1)
        prior_t = rng.choice([-1.0] + tvals)
        prior_rec = -1 if prior_t < 0 else 10_000
        assert pooled(ts, prior_t, prior_rec, k0, rng, run) == reference_loop(ts, prior_t, prior_rec, k0)


def test_the_model_has_teeth():
    """Taking an equal t from a later run (<= instead of <) would change results: the model sees it."""
    rng = random.Random(7)
    differs = 0
    for _ in range(2000):
        n = rng.randint(2, 40)
        ts = [rng.choice([1.0, 2.0]) if rng.random() < 0.5 else None for _ in range(n)]
        want = reference_loop(ts, -1.0, -1, 0)
        hits = [(t, p) for p, t in enumerate(ts) if t is not None]
        if hits:
            last_min = max(p for t, p in hits if t == min(hits)[0])
            differs += (min(hits)[0], last_min) != want
    assert differs > 100

"""The brute-force replay's skipped leaf boxes (pt_wavefront.hip bf_replay_stackless, round 4): a leaf
child's box test — the reference's `li`/`ri` (src/wgsl-util/intersection-logic.wgsl:39-42) — is
computed only while the leaf holds a hit entry the ray has not tested yet, and an unneeded leaf is
taken as not hit.  Claim: the replay's result (closest record and t) is unchanged, ties included.

A host model of the replay, step for step as the kernel has it — pending set in pre-order (right
subtree first), mailbox set `tested`, phase 1's hit set and t per uid, strict-< updates with the
pair's tie-break (mb_first_node: the first of the pair's two entries in the reference's leaf order,
left leaf then right), exit-distance pruning of internal children, the tmin early exit — run with
and without the skip on random trees, leaf contents (uids repeated across leaves, as the
reference's duplicating builder makes them), hit sets with forced equal t's and random box
distances.  Host logic, no GPU."""
import random

import pytest

from test_replay_order import preorder_right_first, random_tree


def make_case(rng):
    children = random_tree(rng, rng.randint(1, 40))
    n_uid = rng.randint(1, 63)
    leaves = {}  # (node, side) -> list of uids in leaf order (a leaf child)
    for n, (l, r) in enumerate(children):
        for side, c in enumerate((l, r)):
            if c is None:
                leaves[(n, side)] = [rng.randrange(n_uid) for _ in range(rng.randint(0, 6))]
    # phase 1: some uids hit, t drawn from a few values so that ties happen
    tvals = [rng.choice([0.5, 1.0, 1.5, 2.0, 3.0]) for _ in range(n_uid)]
    hits = {u for u in range(n_uid) if rng.random() < 0.35}
    boxes = {}  # (node, side) -> box distance (<= 0: missed)
    for n in range(len(children)):
        for side in (0, 1):
            boxes[(n, side)] = rng.choice([-1.0, 0.25, 0.75, 1.25, 1.75, 2.5, 4.0])
    return children, leaves, tvals, hits, boxes


def subtree_uids(children, leaves):
    """uid union below each internal node (BfNode's subtree masks, pt_capi.hip build_layout)."""
    memo = {}

    def rec(n):
        if n not in memo:
            u = set()
            for side, c in enumerate(children[n]):
                u |= rec(c) if c is not None else set(leaves.get((n, side), []))
            memo[n] = u
        return memo[n]
    for n in range(len(children)):
        rec(n)
    return memo


def replay(case, skip, skip_subtrees=False):
    children, leaves, tvals, hits, boxes = case
    pre, order = preorder_right_first(children)
    sub = subtree_uids(children, leaves)
    tmin = min((tvals[u] for u in hits), default=3.0e38)
    if not hits:
        return -1, -1.0
    pend, tested, best, best_t = 1, set(), -1, -1.0
    while pend:
        i = (pend & -pend).bit_length() - 1
        pend &= pend - 1
        n = order[i]
        l, r = children[n]
        lint, rint = l is not None, r is not None
        lleaf, rleaf = leaves.get((n, 0), []), leaves.get((n, 1), [])
        if skip:
            lneed = lint or bool((set(lleaf) & hits) - tested)
            rneed = rint or bool((set(rleaf) & hits) - tested)
        else:
            lneed = rneed = True
        ld = boxes[(n, 0)] if lneed else -1.0
        rd = boxes[(n, 1)] if rneed else -1.0
        li, ri = lneed and ld > 0.0, rneed and rd > 0.0
        m = (set(lleaf) if (li and not lint) else set()) | (set(rleaf) if (ri and not rint) else set())
        rh = sorted((m - tested) & hits)  # uid order (ctz)
        tested |= m
        pair = (lleaf if (li and not lint) else []) + (rleaf if (ri and not rint) else [])  # reference order
        bcur = False
        for u in rh:
            t = tvals[u]
            take = best_t < 0.0 or t < best_t
            if t == best_t and bcur:  # mb_first_node: which of u, best comes first in the pair
                first = next(x for x in pair if x in (u, best))
                take = first == u
            if take:
                best_t, best, bcur = t, u, True
        if best_t == tmin:
            pend = 0
        else:
            tl = li and lint and not (best_t > 0.0 and ld > best_t)
            tr = ri and rint and not (best_t > 0.0 and rd > best_t)
            if skip_subtrees:  # a subtree without an untested hit entry cannot change best
                tl = tl and bool((sub[l] & hits) - tested)
                tr = tr and bool((sub[r] & hits) - tested)
            if tl:
                pend |= 1 << pre[l]
            if tr:
                pend |= 1 << pre[r]
    return best, best_t


@pytest.mark.parametrize("seed", range(200))
def test_skipping_unneeded_leaf_boxes_changes_nothing(seed):
    rng = random.Random(seed)
    for _ in range(50):
        case = make_case(rng)
        want = replay(case, False)
        assert replay(case, True) == want
        assert replay(case, True, skip_subtrees=True) == want  # and whole subtrees without one


def test_the_model_has_teeth():
    """Dropping a NEEDED leaf (one with an untested hit) would change results: the model sees it."""
    rng = random.Random(3)
    differs = 0
    for _ in range(400):
        children, leaves, tvals, hits, boxes = make_case(rng)
        # hide every leaf that holds a hit (what a wrong skip rule would do)
        hidden = {k: ([] if set(v) & hits else v) for k, v in leaves.items()}
        a = replay((children, leaves, tvals, hits, boxes), True)
        b = replay((children, hidden, tvals, hits, boxes), True)
        differs += a != b
    assert differs > 50

"""The brute-force replay's stackless walk (pt_wavefront.hip bf_replay_stackless) visits the same
nodes in the same order as the reference's stack walk (program-raymarch.wgsl traversal, restated
by lean_decide: right child first, the left one stacked when both are taken), for any
decisions — the claim its comment makes.  Internal nodes are numbered in pre-order, right
subtree first (pt_capi.hip build_layout), and the pending set is walked smallest number first.
Checked on random trees with random, history-dependent decisions (host logic, no GPU)."""
import random

import pytest


def random_tree(rng, n_internal):
    """children[i] = (left, right), each an internal node index or None (a leaf)."""
    children = [[None, None]]
    free = [(0, 0), (0, 1)]
    while len(children) < n_internal:
        p, side = free.pop(rng.randrange(len(free)))
        children[p][side] = len(children)
        children.append([None, None])
        free += [(len(children) - 1, 0), (len(children) - 1, 1)]
    return children


def preorder_right_first(children):
    pre, order, st = {}, [], [0]
    while st:
        n = st.pop()
        pre[n] = len(order)
        order.append(n)
        l, r = children[n]
        if l is not None:
            st.append(l)
        if r is not None:
            st.append(r)
    return pre, order


def stack_walk(children, decide):
    seq, st, node = [], [], 0
    while True:
        seq.append(node)
        l, r = children[node]
        tl, tr = decide(node, len(seq))
        tl, tr = tl and l is not None, tr and r is not None
        if tl and tr:
            st.append(l)
            node = r
        elif tr:
            node = r
        elif tl:
            node = l
        elif st:
            node = st.pop()
        else:
            return seq


def stackless_walk(children, decide):
    pre, order = preorder_right_first(children)
    seq, pend = [], 1
    while pend:
        i = (pend & -pend).bit_length() - 1
        pend &= pend - 1
        node = order[i]
        seq.append(node)
        l, r = children[node]
        tl, tr = decide(node, len(seq))
        if tl and l is not None:
            pend |= 1 << pre[l]
        if tr and r is not None:
            pend |= 1 << pre[r]
    return seq


@pytest.mark.parametrize("seed", range(40))
def test_stackless_walk_matches_stack_walk(seed):
    rng = random.Random(seed)
    children = random_tree(rng, rng.randint(1, 64))
    salt = rng.random()

    def decide(node, step):  # depends on the node and on how far the walk has gone (closest t so far)
        h = random.Random(hash((node, step, salt)))
        return h.random() < 0.7, h.random() < 0.7

    assert stackless_walk(children, decide) == stack_walk(children, decide)


def test_every_node_when_nothing_is_pruned():
    rng = random.Random(1)
    children = random_tree(rng, 64)
    seq = stackless_walk(children, lambda n, s: (True, True))
    pre, order = preorder_right_first(children)
    assert seq == order and len(seq) == 64

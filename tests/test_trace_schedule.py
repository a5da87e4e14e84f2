"""CPU model of k_wf_trace's work split and write-back (pt_wavefront.hip), step for step.

Wave w of N takes the queue windows w, w+N, ...; idle lanes take entries of the window in LDS
(ballot rank order); a window is written back from the hit ring once all its entries were handed
out and traced; the next window enters only while the ring has room.  The model checks the
invariants the kernel relies on — every entry traced and written back exactly once, with its own
record, and every wave terminates — for adversarial traversal lengths (all 1: the whole window
finishes at once, which is what exposed a flush that ran ahead of the window in LDS).
"""
import random

import pytest

WIN, RING, LANES = 32, 128, 64


def run_wave(count, nwaves, w, lengths, seed, max_iters=10**6):
    rnd = random.Random(seed)
    nwin = (count + WIN - 1) // WIN
    if w >= nwin:
        return []
    J = (nwin - w + nwaves - 1) // nwaves

    def wbase(j):
        return (w + j * nwaves) * WIN

    def wcount(j):
        return min(WIN, count - wbase(j))

    jl, wv = 0, wcount(0)
    nv = wcount(1) if J > 1 else 0
    cur = flushed = 0
    has, sq, left = [False] * LANES, [0] * LANES, [0] * LANES
    ring, out = {}, []
    for _ in range(max_iters):
        while flushed < J * WIN:  # write back complete windows
            jf = flushed // WIN
            handed = jf < jl or (jf == jl and cur == jl * WIN + wv)
            if not handed or any(has[l] and sq[l] < flushed + WIN for l in range(LANES)):
                break
            for l in range(wcount(jf)):
                out.append((wbase(jf) + l, ring.pop((flushed + l) % RING)))
            flushed += WIN
        need = [not h for h in has]
        if any(need):
            if cur == jl * WIN + wv and jl + 1 < J and (jl + 2) * WIN - flushed <= RING:
                jl, wv, cur = jl + 1, nv, (jl + 1) * WIN
                if jl + 1 < J:
                    nv = wcount(jl + 1)
            wend = jl * WIN + wv
            if cur < wend:
                rank = 0
                for l in range(LANES):
                    if need[l]:
                        k = cur + rank
                        rank += 1
                        if k < wend:
                            sq[l], has[l], left[l] = k, True, rnd.choice(lengths)
                cur = min(cur + rank, wend)
        if not any(has):
            if jl + 1 >= J and cur == jl * WIN + wv and flushed >= J * WIN:
                return out
            continue
        for l in range(LANES):  # one traversal step
            if has[l]:
                left[l] -= 1
                if left[l] == 0:
                    slot = sq[l] % RING
                    assert slot not in ring, "hit ring overwritten before write-back"
                    ring[slot] = wbase(sq[l] // WIN) + sq[l] % WIN
                    has[l] = False
    raise AssertionError(f"wave {w} did not terminate (count={count}, nwaves={nwaves})")


@pytest.mark.parametrize("lengths", [[1], [1, 2], [1, 2, 3, 5, 40, 200]])
@pytest.mark.parametrize("count,nwaves", [(1, 1), (31, 2), (32, 1), (33, 3), (1000, 8), (4095, 8), (20000, 64),
                                          (100003, 8)])
def test_every_entry_traced_once_and_written_back(count, nwaves, lengths):
    out = []
    for w in range(nwaves):
        out += run_wave(count, nwaves, w, lengths, seed=count * 31 + w)
    assert sorted(e for e, _ in out) == list(range(count))
    assert all(e == rec for e, rec in out)

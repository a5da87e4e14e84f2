"""CPU model of the region-partitioned queues of the fused kernel (pt_wavefront.hip: k_wf_generate's
region layout and closed-form counts, k_wf_step_bf's regions; the host's rstride
and queue slack in pt_capi.hip / pt_kernels.h), step for step.

64-path batch j of P paths goes to region j % R at offset (j // R) * 64 + p % 64 of that region;
region r holds rstride = qcap // R // 64 * 64 entries, qcap = the queue entries of the half (the
batch's capacity plus the slack 2 * kQueueSlackRegions * 64, halved for the dual-stream halves).
Checks, for adversarial P and R: every path lands in exactly one slot, inside its region; the
kernel's closed-form count of each region equals the real count; and a region can hold its paths
(the survivors of a region never exceed its input, so that bounds every later iteration too).
"""
import numpy as np
import pytest

K_REGIONS, K_SLACK = 512, 4096


def closed_form_count(r, P, R):
    """k_wf_generate / k_wf_step_bf (GEN): count of region r."""
    nbat = (P + 63) // 64
    n = (nbat - r + R - 1) // R if r < nbat else 0
    if n == 0:
        return 0
    last = r + (n - 1) * R
    tail = 64 - (P & 63) if (last == nbat - 1 and (P & 63)) else 0
    return n * 64 - tail


def layout(P, R, rstride):
    p = np.arange(P, dtype=np.int64)
    j = p // 64
    region = j % R
    off = (j // R) * 64 + (p & 63)
    return region, off, region * rstride + off


@pytest.mark.parametrize("capacity", [4096, 1 << 20, 2073600, 8 << 20])
@pytest.mark.parametrize("dual", [False, True])
@pytest.mark.parametrize("R", [1, 3, 64, 24, K_REGIONS])
def test_region_layout_fits_and_counts(capacity, dual, R):
    qn = capacity + 2 * K_SLACK * 64
    qcap = qn // 2 if dual else qn
    rstride = qcap // R // 64 * 64
    Pmax = capacity // 2 if dual else capacity
    for P in sorted({1, 63, 64, 65, Pmax - 1, Pmax} - {0}):
        if P > Pmax or P <= 0:
            continue
        region, off, idx = layout(P, R, rstride)
        assert off.max() < rstride                          # inside its region
        assert idx.max() < qcap                             # inside the half's queue arrays
        assert len(np.unique(idx)) == P                     # one slot per path
        counts = np.bincount(region, minlength=R)
        for r in list(range(min(R, 70))) + [R - 1]:
            assert closed_form_count(r, P, R) == counts[r], (P, R, r)
        # the region's entries are its first count_r slots (the kernels read b * 64 + lane < count)
        for r in {0, R - 1}:
            mine = np.sort(off[region == r])
            assert np.array_equal(mine, np.arange(counts[r]))


@pytest.mark.parametrize("R", [1, 3, 64, K_REGIONS])
@pytest.mark.parametrize("P", [1, 63, 64, 65, 4096 + 17, 2 * 1024 * 1024])
def test_gen_path_index_inverts_the_layout(P, R):
    """k_wf_step_bf's GEN launch makes path p = (b * R + rg) * 64 + lane for in-region batch b,
    lane < count_rg - b * 64: exactly the path k_wf_generate would have stored at region rg,
    offset b * 64 + lane — every path once, in the same slot."""
    region, off, _ = layout(P, R, 1 << 40)
    b, lane = off // 64, off % 64
    p = np.arange(P, dtype=np.int64)
    assert np.array_equal((b * R + region) * 64 + lane, p)
    for rg in {0, R - 1, min(R - 1, 5)}:
        n = closed_form_count(rg, P, R)
        slots = np.arange(n)
        made = (slots // 64 * R + rg) * 64 + slots % 64
        assert np.array_equal(np.sort(p[region == rg]), made)
        assert made.size == 0 or made.max() < P

"""The relief pair's workgroup map (csrc/bb_pairmap.h, CPU host build).

relief_pair1_kernel is persistent: its teams take envs from rings per (kind, XCD label)
and spin until every env is done.  A (kind, label) whose workgroups are not resident would
leave its ring undrained, so the map interleaves the kinds by groups of 8 blocks (one per
label): any resident prefix of the grid of at least 16 blocks serves every ring.  These
checks cover the splits pair_adapt_kernel and bb_create can produce (multiples of 8, at
least cap/8 per kind) on the 1024-workgroup grid of a 256-CU MI355X and smaller grids.
"""
import pytest

import hostcheck_lib as H


def _splits(cap):
    G = cap // 8
    lo = (G + 7) // 8
    return [((G - gs) * 8, gs * 8) for gs in sorted({lo, lo + 1, G // 3, G // 2, G - lo - 1, G - lo}) if lo <= gs <= G - lo]


@pytest.mark.parametrize("cap", [1024, 512, 128])
def test_pair_map_is_a_bijection_per_kind(cap):
    for nf, ns in _splits(cap):
        seen = {0: set(), 1: set()}
        for b in range(cap + 16):
            k, wg = H.pair_kind_of(b, nf, ns)
            if b >= nf + ns:
                assert k == -1
                continue
            assert k in (0, 1) and wg % 8 == b % 8  # the block's XCD label is its ring label
            assert wg not in seen[k]
            seen[k].add(wg)
        assert seen[0] == set(range(nf)) and seen[1] == set(range(ns)), (nf, ns)


@pytest.mark.parametrize("cap", [1024, 512, 128])
def test_every_resident_prefix_serves_every_ring(cap):
    """Blocks 0..15 already hold a fast and a full workgroup of every label, and kinds stay
    interleaved: no run of full-kind (or fast-kind) groups longer than the split requires."""
    for nf, ns in _splits(cap):
        kinds = [H.pair_kind_of(b, nf, ns)[0] for b in range(nf + ns)]
        for p in (16, 24, 64, nf + ns):
            have = {(kinds[b], b % 8) for b in range(p)}
            assert have == {(k, x) for k in (0, 1) for x in range(8)}, (nf, ns, p)
        groups = kinds[::8]
        assert all(len(set(kinds[8 * g:8 * g + 8])) == 1 for g in range(len(groups)))
        G, gmin = (nf + ns) // 8, min(nf, ns) // 8
        bound = -(-(G - 2) // max(gmin - 1, 1)) + 1  # groups 0 and 1 are fixed, the rest centred
        run = longest = 0
        for i, k in enumerate(groups):
            run = run + 1 if i and k == groups[i - 1] else 1
            longest = max(longest, run)
        assert longest <= bound, (nf, ns, longest, bound)


def test_solo_workgroups_leave_every_label_a_full_workgroup():
    """BB_PAIR_SOLO is clamped to cap/8 - 8 (bb_create): the solo workgroups are the first
    full-kind indices, and at the adapt floor (cap/8 full workgroups) the rest still cover
    all 8 labels."""
    cap = 1024
    nsolo = cap // 8 - 8
    for nf, ns in _splits(cap):
        labels = set()
        for b in range(nf + ns):
            k, wg = H.pair_kind_of(b, nf, ns)
            if k == 1 and wg >= nsolo:
                labels.add(b % 8)
        assert labels == set(range(8)), (nf, ns)

"""The FAST cardinal pre-test of mcs_orb_level (csrc/mcs_orb_core.h orb_fast_pretest) is a
necessary condition of the segment test (orb_fast_test): every brighter / darker mask with an arc
of 9 contiguous circle positions passes it, so filtering with it changes no keypoint.  Exhaustive
over the 2^16 masks, with the two functions' bit formulas restated here."""
import numpy as np


def _segment(m):
    """orb_fast_test's run-of-9 search on one 16-bit mask (doubled to 32 bits)."""
    a32 = m | (m << 16)
    a = a32 & (a32 >> 1)
    a &= a >> 2
    a &= a >> 4
    a &= a32 >> 8
    return (a & 0xFFFF) != 0


def _pretest(m):
    """orb_fast_pretest on the cardinal bits 0, 4, 8, 12 of the same mask."""
    c = ((m >> 0) & 1) | ((m >> 4) & 1) << 1 | ((m >> 8) & 1) << 2 | ((m >> 12) & 1) << 3
    r = c & ((c >> 1) | (c << 3))
    return (r & 15) != 0


def test_pretest_is_necessary_for_every_mask():
    m = np.arange(1 << 16, dtype=np.int64)
    seg = _segment(m)
    pre = _pretest(m)
    assert seg.sum() > 0
    assert not np.any(seg & ~pre)          # every segment-test pass also passes the pre-test
    assert pre.sum() < (1 << 16)           # and the pre-test does reject masks


def test_segment_formula_matches_arc_definition():
    m = np.arange(1 << 16, dtype=np.int64)
    bits = (m[:, None] >> np.arange(16)) & 1
    ring = np.concatenate([bits, bits], axis=1)
    arcs = np.stack([ring[:, s:s + 9].all(axis=1) for s in range(16)], axis=1).any(axis=1)
    assert np.array_equal(arcs, _segment(m))

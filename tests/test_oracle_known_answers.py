"""Known-answer tests of the CPU oracle (OpenCV 3.4 warpPerspective restated).

OpenCV is not installed here or on the GPU box and the reference ships no images, so these pin
the restatement against hand-derived answers and against a second, independent pure-Python
restatement of the same operation order.
"""
import math

import numpy as np
import pytest

from oracle import oracle


def py_invert(m):
    """cv::invert(DECOMP_LU) closed form for 3x3 doubles, in pure Python floats."""
    m = [float(v) for v in np.asarray(m, np.float64).reshape(9)]
    M = lambda i, j: m[i * 3 + j]  # noqa: E731
    d = (M(0, 0) * (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) -
         M(0, 1) * (M(1, 0) * M(2, 2) - M(1, 2) * M(2, 0)) +
         M(0, 2) * (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)))
    if d == 0.0:
        return [0.0] * 9
    d = 1.0 / d
    return [(M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) * d,
            (M(0, 2) * M(2, 1) - M(0, 1) * M(2, 2)) * d,
            (M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1)) * d,
            (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * d,
            (M(0, 0) * M(2, 2) - M(0, 2) * M(2, 0)) * d,
            (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * d,
            (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * d,
            (M(0, 1) * M(2, 0) - M(0, 0) * M(2, 1)) * d,
            (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * d]


def py_round_clamped(v):
    v = v if v < 2147483647.0 else 2147483647.0
    v = v if -2147483648.0 < v else -2147483648.0
    return int(round(v))   # Python round() is round-half-to-even


def py_map(Mi, bilinear, xb, x1, y):
    """WarpPerspectiveInvoker arithmetic for pixel xb + x1 of row y (pure Python doubles)."""
    X0 = Mi[0] * xb + Mi[1] * y + Mi[2]
    Y0 = Mi[3] * xb + Mi[4] * y + Mi[5]
    W0 = Mi[6] * xb + Mi[7] * y + Mi[8]
    W = W0 + Mi[6] * x1
    if bilinear:
        W = 32.0 / W if W else 0.0
    else:
        W = 1.0 / W if W else 0.0
    return (py_round_clamped((X0 + Mi[0] * x1) * W), py_round_clamped((Y0 + Mi[3] * x1) * W))


def random_homographies(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        th = rng.uniform(-0.3, 0.3)
        s = rng.uniform(0.8, 1.25)
        H = np.array([[s * math.cos(th), -s * math.sin(th), rng.uniform(-300, 300)],
                      [s * math.sin(th), s * math.cos(th), rng.uniform(-100, 100)],
                      [rng.uniform(-4e-4, 4e-4), rng.uniform(-4e-4, 4e-4), 1.0]])
        out.append(H)
    return out


def test_invert_matches_python_restatement_bitwise():
    for H in random_homographies(200, 1):
        got = oracle.invert3x3(H).reshape(9)
        want = py_invert(H)
        assert [float(v) for v in got] == want
        assert np.allclose(got.reshape(3, 3) @ H, np.eye(3), atol=1e-9)


def test_invert_singular_is_zero():
    assert (oracle.invert3x3(np.ones((3, 3))) == 0).all()


def test_bilinear_table_entries():
    for fy in range(32):
        for fx in range(32):
            w = oracle.bilinear_weights(fx, fy).astype(np.int64)
            if fx == 0 and fy == 0:
                # saturate_cast<short>(1.0 * 32768) = 32767, the fix-up lands on w11
                assert list(w) == [32767, 0, 0, 1]
                continue
            assert list(w) == [32 * (32 - fx) * (32 - fy), 32 * fx * (32 - fy),
                               32 * (32 - fx) * fy, 32 * fx * fy]
            assert w.sum() == 32768


def test_table_quirk_equals_exact_weights_for_u8():
    """The (0,0) entry {32767,0,0,1} gives p00 for every u8 pair: the GPU's exact {32768,0,0,0}
    weights are therefore output-identical."""
    p = np.arange(256, dtype=np.int64)
    p00, p11 = np.meshgrid(p, p, indexing="ij")
    quirk = (32767 * p00 + p11 + 16384) >> 15
    exact = (32768 * p00 + 16384) >> 15
    assert (quirk == exact).all() and (exact == p00).all()


@pytest.mark.parametrize("bilinear", [True, False])
def test_map_pixel_matches_independent_python(bilinear):
    interp = oracle.INTER_LINEAR if bilinear else oracle.INTER_NEAREST
    rng = np.random.default_rng(7)
    for H in random_homographies(40, 2):
        Mi = py_invert(H)
        for _ in range(50):
            xb = int(rng.integers(0, 100)) * 64
            x1 = int(rng.integers(0, 64))
            y = int(rng.integers(0, 2000))
            X, Y = oracle.map_pixel(np.array(Mi), interp, xb, x1, y)
            wx, wy = py_map(Mi, bilinear, xb, x1, y)
            if bilinear:
                # the oracle reports (sx*32 + fx): sx = X >> 5 saturated to int16, fx = X & 31
                sat = lambda v: max(-32768, min(32767, v >> 5)) * 32 + (v & 31)  # noqa: E731
                assert (X, Y) == (sat(wx), sat(wy))
            else:
                assert (X, Y) == (max(-32768, min(32767, wx)), max(-32768, min(32767, wy)))


def test_block_start_evaluation_is_not_the_naive_formula():
    """X0 is evaluated at the 64-column block start (OpenCV order): X = rint(32*((M0*xb + M2) +
    M0*x1)), not rint(32*(M0*x + M2)).  Rounding differences only matter next to a .5 tie, so the
    matrices are built to land pixel 65 on a tie; the oracle must follow the block form."""
    rng = np.random.default_rng(11)
    found = 0
    for _ in range(4000):
        M0 = float(rng.uniform(0.5, 2.0))
        k = int(rng.integers(100, 5000))
        t = (k + 0.5) / 32.0
        M2 = t - M0 * 65
        Mi = [M0, 0.0, M2, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0]
        blk = py_map(Mi, True, 64, 1, 0)
        naive = py_map(Mi, True, 65, 0, 0)
        if blk != naive:
            found += 1
            assert oracle.map_pixel(np.array(Mi), oracle.INTER_LINEAR, 64, 1, 0) == blk
    assert found > 10


def test_round_half_even_ties():
    # inverse map M: fX = (x/64) * 32 = x/2 exactly -> ties at odd x
    M = np.array([[1 / 64, 0, 0], [0, 0, 0], [0, 0, 1]], np.float64)
    got = [oracle.map_pixel(M, oracle.INTER_LINEAR, 0, x, 0)[0] for x in (1, 3, 5, 7)]
    assert got == [0, 2, 2, 4]


def _checker(h, w, c=3, seed=0):
    rng = np.random.default_rng(seed)
    return rng.integers(1, 256, size=(h, w, c), dtype=np.uint8)


@pytest.mark.parametrize("tx,ty", [(7, 3), (-5, 11), (0, 0), (40, -2)])
def test_integer_translation_nearest_equals_bilinear_equals_copy(tx, ty):
    src = _checker(30, 50)
    H = np.array([[1, 0, tx], [0, 1, ty], [0, 0, 1]], np.float64)
    dw, dh = 70, 45
    lin = oracle.warp_perspective(src, H, (dw, dh), oracle.INTER_LINEAR)
    nn = oracle.warp_perspective(src, H, (dw, dh), oracle.INTER_NEAREST)
    want = np.zeros((dh, dw, 3), np.uint8)
    for y in range(dh):
        for x in range(dw):
            sx, sy = x - tx, y - ty
            if 0 <= sx < 50 and 0 <= sy < 30:
                want[y, x] = src[sy, sx]
    assert (lin == want).all() and (nn == want).all()


@pytest.mark.parametrize("k", [1, 5, 16, 31])
def test_subpixel_shift_known_taps(k):
    """Forward shift by k/32 px: taps x-1 and x with weights 1024k and 1024(32-k)."""
    src = _checker(8, 40, 1)[..., 0]
    H = np.array([[1, 0, k / 32], [0, 1, 0], [0, 0, 1]], np.float64)
    out = oracle.warp_perspective(src, H, (40, 8), oracle.INTER_LINEAR)
    p = src.astype(np.int64)
    for x in range(1, 40):
        want = (p[:, x - 1] * 1024 * k + p[:, x] * 1024 * (32 - k) + 16384) >> 15
        assert (out[:, x] == want).all()
    # x = 0: the left tap (x-1 = -1) is outside and reads the border value 0
    want0 = (p[:, 0] * 1024 * (32 - k) + 16384) >> 15
    assert (out[:, 0] == want0).all()


def test_fully_outside_is_black():
    src = _checker(10, 10)
    H = np.array([[1, 0, 500], [0, 1, 500], [0, 0, 1]], np.float64)
    assert (oracle.warp_perspective(src, H, (30, 20)) == 0).all()


def test_zero_w_maps_to_origin():
    """W == 0 -> the inverse-mapped coordinate is (0, 0) for every pixel."""
    src = _checker(6, 6)
    Mi = np.array([[1, 2, 3], [4, 5, 6], [0, 0, 0]], np.float64)
    out = oracle.warp_perspective(src, Mi, (9, 5), oracle.INTER_LINEAR, inverse_map=True)
    assert (out == src[0, 0]).all()


def test_narrow_canvas_block_width():
    """Canvases narrower than 64 columns or shorter than 16 rows change the block width
    (bw0 = min(1024 / min(16, H), W)); the warp must still equal the pure-Python restatement."""
    src = _checker(12, 20)
    H = np.array([[1.03, 0.02, 2.3], [-0.01, 0.98, 1.7], [2e-3, 1e-3, 1.0]], np.float64)
    for dw, dh in [(30, 9), (200, 5), (17, 40)]:
        out = oracle.warp_perspective(src, H, (dw, dh))
        Mi = py_invert(H)
        bh0 = min(16, dh)
        bw0 = min(1024 // bh0, dw)
        for y in range(dh):
            for x in range(dw):
                X, Y = py_map(Mi, True, (x // bw0) * bw0, x % bw0, y)
                assert oracle.map_pixel(np.array(Mi), 1, (x // bw0) * bw0, x % bw0, y) == (X, Y)
        assert out.shape == (dh, dw, 3)

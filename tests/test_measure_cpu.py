"""Post-detection measurement, CPU side: the fp64 restatement of
motionParaMeasure.m (oracle/measure_ref.py) pinned against independent implementations of
the builtins it stands on, the reference's edge re-anchoring semantics, and the calibration
tables of angle_KvalueGen.m / freValueGen.m.

Parity of the restatement itself is unpinned (the reference ships no measurement outputs);
what is pinned: MATLAB's interp1 'spline' = not-a-knot cubic spline (scipy CubicSpline, an
independent implementation of that published definition), MATLAB's colon a:d:b, find()
column-major order, and known-answer peaks (a sampled parabola, and a Gaussian whose true maximum is known).
"""
import numpy as np
import pytest

import measure_ref as mr


@pytest.mark.parametrize("n", [5, 7, 9, 4, 6])
def test_spline_matches_scipy_not_a_knot(n):
    from scipy.interpolate import CubicSpline
    rng = np.random.default_rng(n)
    y = rng.standard_normal(n) * 3 + 10
    m = mr.spline_m(y)
    cs = CubicSpline(np.arange(n, dtype=np.float64), y, bc_type="not-a-knot")
    t = np.linspace(0, n - 1, 8 * (n - 1) + 1)
    got = np.array([mr.spline_eval(y, m, ti) for ti in t])
    np.testing.assert_allclose(got, cs(t), rtol=0, atol=1e-12)
    np.testing.assert_allclose(m, cs(np.arange(n), 2), rtol=0, atol=1e-11)


def test_spline_three_points_is_the_parabola():
    y = np.array([1.0, 4.0, 2.5])
    m = mr.spline_m(y)
    coef = np.polyfit([0, 1, 2], y, 2)
    t = np.linspace(0, 2, 17)
    np.testing.assert_allclose([mr.spline_eval(y, m, ti) for ti in t], np.polyval(coef, t), atol=1e-13)


@pytest.mark.parametrize("a,k,b", [(1.0, 8, 5.0), (3.0, 4, 7.0), (100.0, 8, 104.0), (1.0, 3, 3.0), (7.0, 64, 15.0)])
def test_colon_matches_matlab(a, k, b):
    q = mr.colon(a, 1.0 / k, b)
    assert len(q) == int(round((b - a) * k)) + 1
    assert q[0] == a and q[-1] == b
    np.testing.assert_allclose(q, np.linspace(a, b, len(q)), atol=1e-12)


def test_fix_cells_reanchoring():
    # inside: unchanged
    assert mr.fix_cells(10, 2, 1, 20) == [8, 9, 10, 11, 12]
    # low edge (:24-27): starts at 1
    assert mr.fix_cells(1, 2, 1, 20) == [1, 2, 3, 4, 5]
    assert mr.fix_cells(2, 2, 1, 20) == [1, 2, 3, 4, 5]
    # high edge (:29-32): ends at R
    assert mr.fix_cells(20, 2, 1, 20) == [16, 17, 18, 19, 20]
    assert mr.fix_cells(19, 2, 1, 20) == [16, 17, 18, 19, 20]
    # velocity (:51-59): lo = M0+2, hi = V-M0
    assert mr.fix_cells(7, 2, 7, 122) == [7, 8, 9, 10, 11]
    assert mr.fix_cells(9, 2, 7, 122) == [7, 8, 9, 10, 11]
    assert mr.fix_cells(122, 2, 7, 122) == [118, 119, 120, 121, 122]
    # a hit deeper in the zeroed rows than extraDots: find() is empty -> MATLAB error
    with pytest.raises(IndexError):
        mr.fix_cells(3, 2, 7, 122)
    with pytest.raises(IndexError):
        mr.fix_cells(126, 2, 7, 122)


def _params(**kw):
    p = dict(extra_dots=2, r_scale=None, delta_r=6.0, r_interp=8, v_scale=None, delta_v=0.25, v_interp=4,
             k_value=10.414385, beam_pos_num=1, beam_angle_step=5.0, ele_comp=0.0, ele_sys_err=0.0, mtd0_num=5)
    p.update(kw)
    return p


def test_known_answer_peak_location():
    """A separable peak exp(-((r-r*)^2/8 + (v-v*)^2/4)) sampled on the grid: the spline
    maxima land within a fraction of the interpolation step of (r*, v*); rEst / vEst follow
    rScale / vScale exactly as motionParaMeasure.m:43,:70 write them."""
    V, R = 128, 200
    r_true, v_true = 73.3, 40.6
    rr, vv = np.meshgrid(np.arange(1, R + 1), np.arange(1, V + 1))
    s = 5.0 * np.exp(-((rr - r_true) ** 2) / 8.0 - ((vv - v_true) ** 2) / 4.0) + 0.01
    d = 0.3 * s
    flag = np.zeros((V, R), np.uint8)
    flag[39, 72] = 1                                   # 1-based (40, 73): the grid maximum
    p = _params(r_scale=np.arange(R) * 6.0 + 12.0, v_scale=3.0 - np.arange(V) * 0.25)
    re, ve, el, cells = mr.motion_para_measure(s, d, flag, **p)
    assert cells.tolist() == [[39, 72]]
    r_cell_max = (re[0] - 12.0) / 6.0 + 1          # rScale(r) + (rCellMax - r)*deltaR, linear rScale
    v_cell_max = (3.0 - ve[0]) / 0.25 + 1           # vScale(fix(v)) - frac*deltaV, linear vScale
    assert abs(r_cell_max - r_true) <= 0.5 / 8 + 0.05
    assert abs(v_cell_max - v_true) <= 0.5 / 4 + 0.1
    assert (r_cell_max * 8) % 1 == pytest.approx(0, abs=1e-9) and (v_cell_max * 4) % 1 == pytest.approx(0, abs=1e-9)
    assert el[0] == pytest.approx(1 * 5.0 + 2.5 - 0.3 * 10.414385, abs=1e-12)


def test_find_order_and_edges():
    """Hits in column-major find() order; edge hits re-anchored; a hit inside the zeroed
    rows deeper than extraDots raises (the reference stops there) or is NaN in the batched
    convention."""
    rng = np.random.default_rng(3)
    V, R = 64, 40
    s = rng.random((V, R)) + 0.5
    d = rng.standard_normal((V, R))
    flag = np.zeros((V, R), np.uint8)
    for v, r in ((10, 5), (3, 5), (30, 0), (63 - 5, 39), (20, 39), (6, 20)):
        flag[v, r] = 1
    p = _params(r_scale=np.arange(R) * 6.0, v_scale=np.linspace(-8, 8, V), mtd0_num=5)
    re, ve, el, cells = mr.motion_para_measure(s, d, flag, on_error="nan", **p)
    assert cells.tolist() == [[30, 0], [3, 5], [10, 5], [6, 20], [20, 39], [58, 39]]
    bad = np.isnan(re)
    # row 3 (1-based 4) is 3 rows inside the zeroed band 1..6 (lo = 7): find() empty -> error
    assert bad.tolist() == [False, True, False, False, False, False]
    with pytest.raises(IndexError):
        mr.motion_para_measure(s, d, flag, **p)


def test_calibration_tables():
    from rsp.measure import angle_KvalueGen, freValueGen
    k1 = angle_KvalueGen(1)
    assert k1.shape == (11, 12)
    assert k1[0, 0] == 10.380672 and k1[3, 11] == 33.493266 and k1[10, 11] == 22.557463
    assert (k1[0] == k1[2]).all() and (k1[3] == k1[4]).all() and (k1[9] == k1[10]).all()
    k2 = angle_KvalueGen(2)
    assert k2[3, 10] == 12.685487 and k2[0, 3] == 9.222804
    assert angle_KvalueGen().tolist() == k1.tolist()
    assert freValueGen(0) == freValueGen(1) == 9365e6
    assert freValueGen(2) == 9375e6 and freValueGen(10) == 9455e6
    with pytest.raises(ValueError):
        freValueGen(11)
    with pytest.raises(ValueError):
        angle_KvalueGen(3)


def test_dmx_scales():
    """DMX_SignalProcessing_main_xzr.m:93-96, :250-253, :313-327: deltaR = c*ts/2, the range
    calibration offsets, deltaV = lambda*prf/N/2, vScale = -lambda*fftshift(f)/2."""
    from rsp import presets
    from rsp.dmx import dmx_scales
    from rsp.measure import freValueGen
    spec = presets.dmx_native(fc=freValueGen(3))
    rS, rL, vS, dR, dV = dmx_scales(spec, 3)
    assert dR == pytest.approx(2.99792458e8 / 12.5e6 / 2)
    assert rS.shape == (62,) and rS[0] == -297.0 and rS[1] - rS[0] == pytest.approx(dR)
    assert rL.shape == (512,) and rL[0] == 62 * 12 - 92.0
    lam = 2.99792458e8 / 9385e6
    assert dV == pytest.approx(lam * (1 / 52.08e-6) / 2048 / 2)
    assert vS.shape == (2048,) and vS[0] == 0 and vS[1] == pytest.approx(-dV) and vS[-1] == pytest.approx(dV)
    assert vS[1024] == pytest.approx(1024 * dV)          # fftshift puts -N/2 at index N/2

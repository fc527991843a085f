"""GPU parity of the post-detection measurement (rsp_motion_measure_dev)
against the fp64 restatement of motionParaMeasure.m (oracle/measure_ref.py).

Bar: bit-exact.  The kernel computes in fp64 with contraction off, in the oracle's operation
order, from the same fp32 sum / diff values (widened exactly), so every estimate, the hit
order (MATLAB's column-major find()) and the hit cells must be identical; hits the reference
stops at with an index error are NaN and counted in count[:, 1].
"""
import numpy as np
import pytest

import measure_ref as mr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def meas():
    import torch
    assert torch.cuda.is_available()
    from rsp.measure import Measure
    m = Measure(0)
    yield m
    m.close()


def _scene(rng, B, V, R, density):
    s = (rng.random((B, V, R)) * 2 + 0.1).astype(np.float32)
    d = (rng.standard_normal((B, V, R)) * 0.5).astype(np.float32)
    f = (rng.random((B, V, R)) < density).astype(np.uint8)
    # edges and the zeroed band: first/last rows and columns, corners
    f[:, 0, 0] = f[:, V - 1, R - 1] = f[:, 0, R - 1] = f[:, V - 1, 0] = 1
    f[:, V // 2, 0] = f[:, V // 2, R - 1] = 1
    return s, d, f


def _kw(e, M0, R, V, rint=8, vint=4):
    return dict(extra_dots=e, r_scale=np.arange(R) * 5.996 + 1.25, delta_r=5.996, r_interp=rint,
                v_scale=-(np.arange(V) - V / 2) * 0.371, delta_v=0.371, v_interp=vint, k_value=10.880367,
                beam_pos_num=5, beam_angle_step=5.0, ele_comp=0.125, ele_sys_err=-0.5, mtd0_num=M0)


def _run(meas, s, d, f, kw, max_hits=None):
    import torch
    p = meas.params(kw["extra_dots"], kw["delta_r"], kw["r_interp"], kw["delta_v"], kw["v_interp"], kw["k_value"],
                    kw["beam_pos_num"], kw["beam_angle_step"], kw["ele_comp"], kw["ele_sys_err"], kw["mtd0_num"])
    est, cells, count = meas.measure_dev(s, d, f, p, kw["r_scale"], kw["v_scale"], max_hits=max_hits)
    torch.cuda.synchronize()
    return est.cpu().numpy(), cells.cpu().numpy(), count.cpu().numpy()


def _check(est, cells, count, s, d, f, kw, cpis=None):
    for b in (range(s.shape[0]) if cpis is None else cpis):
        re, ve, el, hc = mr.motion_para_measure(s[b].astype(np.float64), d[b].astype(np.float64), f[b],
                                                on_error="nan", **kw)
        n = len(re)
        assert count[b, 0] == n
        assert count[b, 1] == int(np.isnan(re).sum())
        w = min(n, est.shape[1])
        assert (cells[b, :w] == hc[:w]).all()
        want = np.stack([re, ve, el], axis=1)[:w]
        got = est[b, :w]
        assert np.array_equal(np.isnan(got), np.isnan(want))
        ok = ~np.isnan(want)
        assert np.array_equal(got[ok], want[ok]), np.abs(got[ok] - want[ok]).max()


@pytest.mark.parametrize("e", [1, 2, 3, 4])
@pytest.mark.parametrize("V,R", [(128, 1024), (64, 250)])   # 4-byte flag words / byte path
def test_measure_parity(meas, e, V, R):
    rng = np.random.default_rng(100 * e + R)
    s, d, f = _scene(rng, 3, V, R, 0.004)
    kw = _kw(e, 5, R, V)
    est, cells, count = _run(meas, s, d, f, kw)
    _check(est, cells, count, s, d, f, kw)
    assert count[:, 0].min() > 20 and count[:, 1].min() >= 1     # the band hits at row 0 / V-1 fail


@pytest.mark.parametrize("V,R", [(64, 256), (96, 250)])
def test_measure_large_batch_path(meas, V, R):
    """batch >= 128: one workgroup per CPI (hits_kernel); smaller batches above run the banded
    path (band_count / band_scan / band_list).  Same bit-exact bar on a sample of CPIs, and
    every CPI's count equals its flag total."""
    rng = np.random.default_rng(V + R)
    s, d, f = _scene(rng, 130, V, R, 0.002)
    kw = _kw(2, 5, R, V)
    est, cells, count = _run(meas, s, d, f, kw)
    assert (count[:, 0] == f.reshape(130, -1).sum(1)).all()
    _check(est, cells, count, s, d, f, kw, cpis=(0, 1, 64, 127, 128, 129))


def test_measure_dense_and_truncated(meas):
    """Many hits per column (several row slices) and max_hits truncation: the count is the
    full hit count, the first max_hits entries are the oracle's first max_hits."""
    V, R = 256, 512
    rng = np.random.default_rng(9)
    s, d, f = _scene(rng, 2, V, R, 0.05)
    kw = _kw(2, 11, R, V, rint=16, vint=2)
    est, cells, count = _run(meas, s, d, f, kw, max_hits=1000)
    assert (count[:, 0] > 1000).all()
    _check(est, cells, count, s, d, f, kw)


def test_measure_empty_and_large_columns(meas):
    """No hits; then one CPI with R > 4096 (several column passes) and a V of 2048 (the DMX
    Doppler size)."""
    V, R = 64, 512
    s = np.ones((1, V, R), np.float32)
    f = np.zeros((1, V, R), np.uint8)
    est, cells, count = _run(meas, s, s, f, _kw(2, 2, R, V))
    assert count.tolist() == [[0, 0]]
    rng = np.random.default_rng(11)
    for V, R in ((32, 8192), (2048, 62)):
        s, d, f = _scene(rng, 1, V, R, 0.002)
        kw = _kw(2, 6, R, V)
        est, cells, count = _run(meas, s, d, f, kw)
        _check(est, cells, count, s, d, f, kw)


def test_motionParaMeasure_mirror(meas):
    """The reference-named single-CPI form: identical series to the oracle; a hit the reference
    cannot re-anchor raises IndexError as the reference stops there."""
    from rsp.measure import angle_KvalueGen
    V, R = 128, 300
    rng = np.random.default_rng(5)
    s, d, f = _scene(rng, 1, V, R, 0.003)
    s, d, f = s[0], d[0], f[0]
    f[:4, :] = 0                                   # 1-based rows 1..4 / V-2..V cannot re-anchor at M0 = 5
    f[V - 3:, :] = 0
    kv = angle_KvalueGen(1)
    rS, vS = np.arange(R) * 6.0, np.linspace(-10, 10, V)
    args = (2, rS, 6.0, 8, vS, 0.2, 4, kv, 3, 5.0, 4, 0.0, 0.0, 5)
    re, ve, el = meas.motionParaMeasure(s, d, f, *args)
    wr, wv, we, _ = mr.motion_para_measure(s.astype(np.float64), d.astype(np.float64), f, 2, rS, 6.0, 8, vS, 0.2, 4,
                                           kv[4, 3], 3, 5.0, 0.0, 0.0, 5)
    assert np.array_equal(re, wr) and np.array_equal(ve, wv) and np.array_equal(el, we)
    f[2, 10] = 1                                   # 1-based row 3: deeper than extraDots into rows 1..6
    with pytest.raises(IndexError):
        meas.motionParaMeasure(s, d, f, *args)


def test_measure_on_dmx_chain(meas):
    """End to end on the DMX two-beam chain (row a8 -> f3): the GPU's own sum / diff / flag
    planes from rsp_pc_mtd_cfar_diff_dev feed the measurement; estimates are bit-exact vs the
    oracle on those planes, and the strongest hit measures the injected target's range."""
    import torch
    from rsp import presets
    from rsp.engine import Engine
    spec = presets.dmx_native()
    eng = Engine(spec, device=0)
    cf = presets.default_cfar(spec)
    rng = np.random.default_rng(1008)
    e = (rng.standard_normal((1, 2, spec.P, spec.R)) + 1j * rng.standard_normal((1, 2, spec.P, spec.R))) \
        * np.sqrt(0.5)
    rep = presets.load_data("refDDCDataMF1").astype(np.complex128).ravel()
    m = np.arange(spec.P)[:, None]
    sig = 0.5 * np.exp(2j * np.pi * 0.11 * m) * rep[None, :] / np.abs(rep).max()
    c0 = 62 + 150
    e[:, 0, :, c0:c0 + rep.size] += sig
    e[:, 1, :, c0:c0 + rep.size] += 0.6 * sig
    d_in = torch.from_numpy(e.astype(np.complex64)).cuda()
    shp = (1, spec.V, spec.R_out)
    d_sum = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_diff = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_sum, diff=d_diff, flag=d_flag, cfar=cf)
    M0 = spec.radar["M0"]
    kw = _kw(2, M0, spec.R_out, spec.V)
    est, cells, count = _run(meas, d_sum, d_diff, d_flag, kw)
    s, d, f = d_sum.cpu().numpy(), d_diff.cpu().numpy(), d_flag.cpu().numpy()
    assert count[0, 0] == f.sum() > 0
    _check(est, cells, count, s, d, f, kw)
    n = count[0, 0]
    amp = s[0][cells[0, :n, 0], cells[0, :n, 1]]
    k = int(np.argmax(amp))
    assert abs(int(cells[0, k, 1]) - (62 + 150)) <= 2     # the long-part range bin of the delay
    eng.close()


def test_dmx_frame_processor(meas):
    """The DMX per-frame loop (DMX_SignalProcessing_main_xzr.m:313-516): chain + measurement of
    the short and the long part, for flag and flagV, over column windows of the same device
    planes.  Each part's series is bit-exact vs the oracle on that part's own matrices (the
    reference measures echo_MTD_sum_short / _long separately, so edge re-anchoring is per
    part), and the strongest long-part hit measures the injected target's range."""
    import torch
    from rsp import presets
    from rsp.dmx import DmxFrameProcessor
    proc = DmxFrameProcessor(freInd=2)
    spec = proc.spec
    rng = np.random.default_rng(77)
    B = 2
    e = (rng.standard_normal((B, 2, spec.P, spec.R)) + 1j * rng.standard_normal((B, 2, spec.P, spec.R))) \
        * np.sqrt(0.5)
    rep = presets.load_data("refDDCDataMF1").astype(np.complex128).ravel()
    m = np.arange(spec.P)[:, None]
    sig = 0.5 * np.exp(2j * np.pi * 0.13 * m) * rep[None, :] / np.abs(rep).max()
    e[:, 0, :, 62 + 200:62 + 200 + rep.size] += sig
    e[:, 1, :, 62 + 200:62 + 200 + rep.size] += 0.7 * sig
    out = proc.process_dev(torch.from_numpy(e.astype(np.complex64)).cuda(), beamPosNum=4)
    torch.cuda.synchronize()
    rS, rL, vS, dR, dV = proc.scales
    s, d = out["sum"].cpu().numpy(), out["diff"].cpu().numpy()
    M0 = spec.radar["M0"]
    kv = proc.kValues[2, 4]
    for fk in ("flag", "flagV"):
        f = out[fk].cpu().numpy()
        for part, (lo, hi), rsc in (("short", (0, 62), rS), ("long", (62, 574), rL)):
            est, cells, count = (t.cpu().numpy() for t in out[(part, fk)])
            kw = dict(extra_dots=2, r_scale=rsc, delta_r=dR, r_interp=8, v_scale=vS, delta_v=dV, v_interp=4,
                      k_value=kv, beam_pos_num=4, beam_angle_step=5.0, ele_comp=0.0, ele_sys_err=0.0, mtd0_num=M0)
            _check(est, cells, count, np.ascontiguousarray(s[:, :, lo:hi]), np.ascontiguousarray(d[:, :, lo:hi]),
                   np.ascontiguousarray(f[:, :, lo:hi]), kw)
    est, cells, count = (t.cpu().numpy() for t in out[("long", "flag")])
    for b in range(B):
        n = count[b, 0]
        assert n > 0
        amp = s[b][cells[b, :n, 0], 62 + cells[b, :n, 1]]
        k = int(np.argmax(amp))
        assert abs(est[b, k, 0] - rL[200]) <= 2 * dR                  # range of the injected delay
    proc.close()

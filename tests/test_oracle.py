"""CPU tests of the oracles (oracle/rsp_ref.py numpy, oracle/rsp_oracle.c C).

Pinning: the reference's one known-answer vector (kaiser_win.mat) plus oracle-independent
known answers: PC peak at the known delay, MTD peak at the known Doppler
bin, CFAR on a constant field = no flags, on a single spike = exactly one flag, edge
fallbacks; and the two independent restatements agreeing with each other.
"""
import numpy as np
import pytest

import coracle
import rsp_ref as ref

DATA = coracle.DATA


def test_kaiser_golden():
    import os
    kw = np.load(os.path.join(os.path.dirname(__file__), "golden", "kaiser_win_1536_beta8.npy"))
    assert kw.shape == (1536,)
    np.testing.assert_allclose(ref.kaiser(1536, 8.0), kw, rtol=0, atol=2e-15)


def test_matlab_builtins():
    assert ref.mround(2.5) == 3 and ref.mround(-2.5) == -3 and ref.mround(0.49) == 0
    # pulse lengths of the v2 chirps = MATLAB colon counts (MTD/fun_MTD_produce.m:61-63)
    p1, p2, p3 = ref.v2_pulses(ref.v2_params())
    assert (len(p1), len(p2), len(p3)) == (4, 200, 700)
    # round(mean(grpdelay(b))) = 17 for the 35-tap symmetric FIR
    assert ref.grpdelay_round_mean(ref.FIR_TAPS_RAW / 511.0) == 17
    # filter(b,1,x): causal, zero state
    y = ref.mfilter(np.array([1.0, 2.0]), np.array([1.0, 0.0, 0.0]))
    np.testing.assert_array_equal(y, [1.0, 2.0, 0.0])
    # fftshift index = numpy fftshift for even and odd lengths
    for P in (8, 9, 64, 1536):
        x = np.arange(P)
        np.testing.assert_array_equal(x[ref.fftshift_index(P)], np.fft.fftshift(x))


@pytest.mark.parametrize("P,div,rows", [(64, 150, (31, 32)), (128, 150, (62, 65)), (256, 150, (125, 130)),
                                        (512, 150, (252, 259)), (128, 20, (57, 70))])
def test_zero_v_rows(P, div, rows):
    # off-centre rows (1-based zv-k .. zv+k)
    assert ref.zero_v_rows(P, div) == rows
    m = ref.fun_0v_pressing(np.ones((P, 3)), div)
    assert np.all(m[rows[0]:rows[1]] == 0) and m.sum() == 3 * (P - (rows[1] - rows[0]))


def test_mtd_zero_num():
    p = ref.v2_params()
    assert [ref.mtd_zero_num(P, p["wavelength"], p["prf"]) for P in (64, 128, 256, 512)] == [2, 5, 11, 22]


def test_pc_known_delay():
    # a lone echo of pulse3 starting at column d of segment 3 compresses to a peak at d
    P, R = 2, 4096
    rp = ref.v2_params(P, R)
    _, p2, p3 = ref.v2_pulses(rp)
    echo = np.zeros((P, R), complex)
    d = 951 + 1000
    echo[:, d:d + 700] = p3
    pc = ref.fun_lss_pulse_compression(echo, p2, p3, 228, 723, R - 951)
    assert int(np.argmax(np.abs(pc[0]))) == d
    assert abs(abs(pc[0, d]) - 700.0) < 1e-9          # |sum |s|^2| = 700
    # the FIR segment: an impulse at n comes out centred at n (circshift by the group delay)
    echo = np.zeros((P, R), complex)
    echo[:, 100] = 1.0
    pc = ref.fun_lss_pulse_compression(echo, p2, p3, 228, 723, R - 951)
    assert int(np.argmax(np.abs(pc[0, :228]))) == 100


def test_mtd_known_doppler():
    P, R = 128, 8
    k = 20                                             # Doppler bin
    m = np.arange(P)
    pc = np.exp(2j * np.pi * k * m / P)[:, None] * np.ones((1, R))
    mtd = ref.fun_Process_MTD(pc)
    # fftshift puts bin k at row k + P/2
    assert np.all(np.argmax(mtd, axis=0) == k + P // 2)


def test_cfar_constant_and_spike():
    V, R = 64, 100
    flat = np.full((V, R), 3.0)
    f, fv = ref.executeCFAR(flat, 5, 7, 5, 0, 5, 7, 5, 0, 2, 1)
    assert f.sum() == 0 and fv.sum() == 0
    spike = flat.copy()
    spike[30, 50] = 100.0
    f, fv = ref.executeCFAR(spike, 5, 7, 5, 0, 5, 7, 5, 0, 2, 1)
    assert f.sum() == 1 and f[30, 50] == 1 and fv[30, 50] == 1
    # edge fallback: a spike in the first used Doppler row still detects (right window used)
    spike = flat.copy()
    spike[3, 50] = 100.0                               # used rows start at M0+1 = 3
    f, fv = ref.executeCFAR(spike, 5, 7, 5, 0, 5, 7, 5, 0, 2, 1)
    assert f[3, 50] == 1 and f.sum() == 1
    # range re-localisation: a Doppler hit moves to the larger neighbour that passes
    row = flat.copy()
    row[30, 50] = 100.0
    row[30, 51] = 200.0
    f, fv = ref.executeCFAR(row, 5, 7, 5, 0, 5, 7, 5, 0, 2, 1)
    assert fv[30, 50] == 1 and fv[30, 51] == 1 and f.sum() == 1 and f[30, 51] == 1
    # too few Doppler cells: MATLAB raises an index error
    with pytest.raises(ref.CfarConfigError):
        ref.executeCFAR(np.ones((20, 40)), 5, 7, 5, 0, 5, 7, 5, 0, 0, 1)


def test_dmx_equivalence():
    # circular correlation via FFT = direct sum with wrap (DMX_SignalProcessing_main_xzr.m:348-352)
    rng = np.random.default_rng(0)
    N = 256
    x = rng.standard_normal((1, N)) + 1j * rng.standard_normal((1, N))
    s = rng.standard_normal(20) + 1j * rng.standard_normal(20)
    H = np.conj(np.fft.fft(s, N))
    y = ref.dmx_pulse_compression(x, 0, N, H)[0]
    direct = np.array([sum(x[0, (n + k) % N] * np.conj(s[k]) for k in range(20)) for n in range(N)])
    np.testing.assert_allclose(y, direct, rtol=0, atol=1e-10)


@pytest.mark.parametrize("name,P,R", [("v2", 64, 1024), ("dmx", 64, 1024), ("legacy", 48, 1031), ("v2", 32, 2048)])
def test_c_oracle_matches_numpy_oracle(name, P, R):
    rng = np.random.default_rng(7)
    echo = rng.standard_normal((2, P, R)) + 1j * rng.standard_normal((2, P, R))
    echo[:, :, :R // 8] += 30.0
    pre = coracle.preset(name, P, R)
    rc = coracle.pc_mtd(echo, pre)
    if name == "v2":
        rn = np.stack([ref.fun_MTD_produce_v2(x, ref.v2_params(P, R)) for x in echo])
    elif name == "dmx":
        rn = np.stack([ref.fun_MTD_produce_dmx_syn(x, np.load(DATA + "/refDDCDataMF1.npy")) for x in echo])
    else:
        rn = np.stack([ref.fun_MTD_produce_legacy(x, np.load(DATA + "/legacy_pulse2.npy"),
                                                  np.load(DATA + "/legacy_pulse3.npy")) for x in echo])
    assert np.linalg.norm(rc - rn) / np.linalg.norm(rn) < 1e-13
    M0 = ref.mtd_zero_num(P, pre["radar"]["wavelength"], pre["radar"]["prf"])
    c = dict(refR=5, saveR=7, TR=4, methodR=0, refV=5, saveV=7, TV=4, methodV=0, M0=M0, rFlag=1, zero_v_div=20)
    fc, fvc = coracle.cfar(rn, c, pre["cfar_segments"])
    segs1 = [(a + 1, b) for a, b in pre["cfar_segments"]]
    for i in range(rn.shape[0]):
        f, fv = ref.main_cfar_chain(rn[i], c, segs1, 20)
        np.testing.assert_array_equal(fc[i], f)
        np.testing.assert_array_equal(fvc[i], fv)
    assert fc.sum() > 0


def test_dmx_mtd_pair_matches_generic_mtd():
    """dmx_mtd_pair = the generic fun_Process_MTD restatement with hamming, nfft 2048 and no
    shift, summed over the beams; the zeroSetFlagMTD rows are 1:M0+1 and end-M0+1:end."""
    rng = np.random.default_rng(3)
    P, R, nfft, m0 = 96, 5, 256, 4
    pl = rng.standard_normal((P, R)) + 1j * rng.standard_normal((P, R))
    pr = rng.standard_normal((P, R)) + 1j * rng.standard_normal((P, R))
    s, d = ref.dmx_mtd_pair(pl, pr, nfft, m0)
    ml = ref.fun_Process_MTD(pl, window=ref.hamming(P), nfft=nfft, shift=False)
    mr = ref.fun_Process_MTD(pr, window=ref.hamming(P), nfft=nfft, shift=False)
    np.testing.assert_allclose(d, mr - ml, rtol=0, atol=1e-9)
    keep = np.ones(nfft, bool)
    keep[:m0 + 1] = False
    keep[nfft - m0:] = False
    np.testing.assert_allclose(s[keep], (ml + mr)[keep], rtol=0, atol=1e-9)
    assert not s[~keep].any() and keep.sum() == nfft - 2 * m0 - 1


@pytest.mark.parametrize("rflag,methodV,methodR,refs", [(1, 0, 0, (5, 7)), (1, 1, 1, (3, 2)), (0, 0, 1, (8, 4)),
                                                        (1, 1, 0, (8, 4))])
def test_c_oracle_near_threshold_mask(rflag, methodV, methodR, refs):
    """The C oracle's near-threshold mask (used at c4/c5 sizes) = the numpy oracle's
    (rsp_ref.executeCFAR(near_tol)), with a tolerance wide enough to mark many cells."""
    ref_n, guard = refs
    rng = np.random.default_rng(11)
    V, R = 96, 700
    rdm = np.abs(rng.standard_normal((2, V, R)) + 1j * rng.standard_normal((2, V, R)))
    rdm[:, 40, 100:103] = [9.0, 14.0, 13.9]
    rdm[:, 60, 400] = 11.0
    c = dict(refR=ref_n, saveR=guard, TR=2.5, methodR=methodR, refV=ref_n, saveV=guard, TV=2.5, methodV=methodV,
             M0=3, rFlag=rflag, zero_v_div=20)
    segs0 = [(0, 250), (250, 700)]
    fc, fvc, ac = coracle.cfar(rdm, c, segs0, near_tol=0.05)
    segs1 = [(a + 1, b) for a, b in segs0]
    for i in range(2):
        f, fv, a = ref.main_cfar_chain(rdm[i], c, segs1, 20, near_tol=0.05)
        np.testing.assert_array_equal(fc[i], f)
        np.testing.assert_array_equal(fvc[i], fv)
        np.testing.assert_array_equal(ac[i], a)
    assert ac.sum() > 50 and fc.sum() > 0


def test_builtins_against_scipy():
    """The oracle's restatements of MATLAB builtins against scipy's: filter(b, 1, x)
    (scipy.signal.lfilter), hamming(n) (symmetric scipy window), kaiser(n, beta), and
    round(mean(grpdelay(b))) (scipy.signal.group_delay of the 35-tap FIR)."""
    sig = pytest.importorskip("scipy.signal")
    rng = np.random.default_rng(5)
    b = ref.FIR_TAPS_RAW / ref.FIR_TAPS_RAW.max()
    x = rng.standard_normal(300) + 1j * rng.standard_normal(300)
    np.testing.assert_allclose(ref.mfilter(b, x), sig.lfilter(b, [1.0], x), rtol=0, atol=1e-12)
    for n in (2, 67, 1536, 2047):
        np.testing.assert_allclose(ref.hamming(n), sig.windows.hamming(n, sym=True), rtol=0, atol=1e-14)
        np.testing.assert_allclose(ref.kaiser(n, 8.0), sig.windows.kaiser(n, 8.0, sym=True), rtol=0, atol=1e-13)
    _, gd = sig.group_delay((b, [1.0]), w=512)
    assert abs(np.mean(gd) - 17.0) < 1e-6
    assert ref.grpdelay_round_mean(b) == int(np.floor(np.mean(gd) + 0.5)) == 17


@pytest.mark.parametrize("name,P,R", [("legacy", 1536, 1031), ("v2", 332, 3404), ("v2", 256, 8192),
                                      ("v2", 512, 16384)])
def test_c_oracle_matches_numpy_oracle_at_checker_sizes(name, P, R):
    """Guard of the large-shape checker: the C oracle (which checks the GPU at the legacy
    native 1536 x 1031 CPI, the v2 native 332 x 3404, c4's 256 x 8192 and c5's 512 x 16384)
    against the loop-faithful numpy oracle on one synthetic CPI of each (SURVEY.md §8d echo),
    fun_MTD_produce + main_cfar's executeCFAR chain with the preset's default CFAR: RDM within
    1e-13, flag and flagV planes identical (executeCFAR.m:21-92, fun_Process_MTD.m:27-37)."""
    from rsp import presets, synth
    spec = presets.make(name, P, R)
    echo = synth.echo_numpy(spec, 1, seed=1200 + P).astype(np.complex128)
    pre = coracle.preset(name, P, R)
    rc = coracle.pc_mtd(echo, pre)
    if name == "v2":
        rn = ref.fun_MTD_produce_v2(echo[0], ref.v2_params(P, R))[None]
    else:
        rn = ref.fun_MTD_produce_legacy(echo[0], np.load(DATA + "/legacy_pulse2.npy"),
                                        np.load(DATA + "/legacy_pulse3.npy"))[None]
    assert np.linalg.norm(rc - rn) / np.linalg.norm(rn) < 1e-13
    cf = presets.default_cfar(spec)
    c = cf.as_dict()
    c["zero_v_div"] = cf.zero_v_div
    fc, fvc = coracle.cfar(rn, c, cf.segments)
    f, fv = ref.main_cfar_chain(rn[0], c, [(a + 1, b) for a, b in cf.segments], cf.zero_v_div)
    np.testing.assert_array_equal(fc[0], f)
    np.testing.assert_array_equal(fvc[0], fv)
    assert f.sum() > 0


def test_range_concate_restatement():
    """fun_lss_range_concate (MatlabProcess_xuzerui/fun_lss_range_concate.m:4-7) keeps MATLAB's
    1-based colons; the preset's 0-based (start, len) parts (what rsp_set_range_concat gathers)
    select the same columns: 1:82, 90:325, 482:1031 -> 868."""
    from rsp import presets
    rng = np.random.default_rng(5)
    s = rng.standard_normal((7, 1031)) + 1j * rng.standard_normal((7, 1031))
    c = ref.fun_lss_range_concate(7, s)
    assert c.shape == (7, 868)
    g = np.concatenate([s[:, a:a + n] for a, n in presets.LEGACY_CONCAT], axis=1)
    assert np.array_equal(c, g)
    assert np.array_equal(c[:, 82], s[:, 89]) and np.array_equal(c[:, 317], s[:, 324])
    assert np.array_equal(c[:, 318], s[:, 481]) and np.array_equal(c[:, 867], s[:, 1030])
    spec = presets.legacy(48, 1031, concat=True)
    assert spec.R_out == 868 and spec.pc_width == 1031 and spec.cfar_segments == [(0, 82), (82, 318), (318, 868)]


def test_pc_and_mtd_restatements_against_direct_sums():
    """Oracle-independent forms of the two transforms (no FFT on the checking side):
    fun_pulse_compression (MTD/fun_pulse_compression.m:10-39, y = ifft(fft(x,N).*fft(h,N)) with
    h = conj(fliplr(s0)), N = len(x)+len(h)-1) against the direct linear convolution; the segment
    cut of fun_lss_pulse_compression (out[n] = y[len(s0)-1+n] = sum_k x[n+k] conj(s0[k])) against
    that correlation sum; and fun_Process_MTD (fun_Process_MTD.m:27-37, |fftshift(fft(col.*kaiser))|)
    against a P x P DFT matrix, the shift as a roll by floor(P/2)."""
    rng = np.random.default_rng(17)
    s0 = rng.standard_normal(37) + 1j * rng.standard_normal(37)
    x = rng.standard_normal(211) + 1j * rng.standard_normal(211)
    y = ref.fun_pulse_compression(s0, x)
    np.testing.assert_allclose(y, np.convolve(x, np.conj(s0[::-1])), rtol=0, atol=1e-11 * np.abs(y).max())
    corr = np.array([np.sum(x[n:n + len(s0)] * np.conj(s0[:len(x[n:n + len(s0)])])) for n in range(len(x))])
    np.testing.assert_allclose(y[len(s0) - 1:len(s0) - 1 + len(x)], corr, rtol=0, atol=1e-11 * np.abs(y).max())
    for P in (16, 48, 128):
        pc = rng.standard_normal((P, 9)) + 1j * rng.standard_normal((P, 9))
        k = np.arange(P)
        dft = np.exp(-2j * np.pi * np.outer(k, k) / P)
        want = np.abs(np.roll(dft @ (pc * ref.kaiser(P, 8.0)[:, None]), P // 2, axis=0))
        np.testing.assert_allclose(ref.fun_Process_MTD(pc), want, rtol=0, atol=1e-11 * want.max())

"""oracle/rsp_ref.py -- TEST INFRASTRUCTURE ONLY.

A loop-faithful fp64 numpy restatement of the MATLAB reference's hot path
(XuZerui2023/Radar-Signal-Process): pulse compression -> MTD -> zero-velocity
suppression -> 2-D CA-CFAR.  It is the *checker* for the HIP product path; nothing
in the product (radar-signal-process_amd/) imports it.  Only tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() may use it.

Pinning: MATLAB/Octave are absent here and on the GPU box, so the
reference cannot be executed.  The oracle is pinned by
  * the reference's one known-answer vector, kaiser_win.mat = kaiser(1536, 8)
    (tests/golden/kaiser_win_1536_beta8.npy), checked in tests/test_oracle.py;
  * oracle-independent known-answer tests (single-target PC peak at the known
    delay, MTD peak at the known Doppler bin, CFAR identities) in tests/;
  * a second, independently written fp64 C restatement (oracle/rsp_oracle.c) that
    uses power-of-two FFT sizes where this file uses MATLAB's exact sizes.
Beyond those, PC / MTD / CFAR *output* parity with MATLAB is "parity unpinned":
no reference test or fixture holds those outputs.

Every function cites the reference file:line it restates.  Paths are relative to
the reference root.  MATLAB semantics reproduced: 1-based
indices, round-half-away-from-zero, colon counts, causal zero-state `filter`,
circshift, fftshift, first-max argmax, `>=` CFAR compare, one-sided edge fallback.
"""
import numpy as np

C_LIGHT = 2.99792458e8

# 35-tap FIR of the short pulse: MTD/fun_lss_pulse_compression.m:31,
# MatlabProcess_xuzerui/fun_lss_pulse_compression.m:21,
# CFAR_WangCai/DMX_SignalProcessing_main_xzr.m:146 (identical integer taps).
FIR_TAPS_RAW = np.array([-9, -7, -2, 10, 27, 40, 42, 24, -13, -57, -89, -86, -30, 77, 220,
                         364, 471, 511, 471, 364, 220, 77, -30, -86, -89, -57, -13, 24, 42,
                         40, 27, 10, -2, -7, -9], dtype=np.float64)


class CfarConfigError(ValueError):
    """The MATLAB code would raise an index error for this shape."""


# ----------------------------------------------------------------------------- builtins
def mround(x):
    """MATLAB round(): half away from zero (numpy rounds half to even)."""
    x = float(x)
    return float(np.sign(x) * np.floor(abs(x) + 0.5))


def colon(a, d, b):
    """MATLAB a:d:b for float arguments (count = floor((b-a)/d) with MATLAB's
    tolerance for an end point that is an integer number of steps away)."""
    q = (b - a) / d
    n = int(np.round(q)) if abs(q - np.round(q)) < 1e-9 * max(1.0, abs(q)) else int(np.floor(q))
    return a + d * np.arange(n + 1, dtype=np.float64)


def kaiser(n, beta):
    """Signal Processing Toolbox kaiser(n, beta) (symmetric)."""
    if n == 1:
        return np.ones(1)
    k = np.arange(n, dtype=np.float64)
    r = (k - (n - 1) / 2.0) / ((n - 1) / 2.0)
    return np.i0(beta * np.sqrt(np.maximum(0.0, 1.0 - r * r))) / np.i0(beta)


def hamming(n):
    """Signal Processing Toolbox hamming(n) (symmetric)."""
    if n == 1:
        return np.ones(1)
    k = np.arange(n, dtype=np.float64)
    return 0.54 - 0.46 * np.cos(2.0 * np.pi * k / (n - 1))


def mfilter(b, x):
    """MATLAB filter(b, 1, x) along the last axis: causal, zero initial state."""
    x = np.asarray(x)
    y = np.zeros(x.shape, dtype=np.result_type(x.dtype, np.float64))
    n = x.shape[-1]
    for k in range(min(len(b), n)):
        y[..., k:] += b[k] * x[..., :n - k]
    return y


def grpdelay_round_mean(b, npts=512):
    """round(mean(grpdelay(b))) as MTD/fun_lss_pulse_compression.m:47 computes it.
    grpdelay's default grid: npts points on [0, pi)."""
    b = np.asarray(b, np.float64)
    w = np.pi * np.arange(npts) / npts
    k = np.arange(len(b))
    e = np.exp(-1j * np.outer(w, k))
    num = e @ (k * b)
    den = e @ b
    ok = np.abs(den) > 1e-12 * np.max(np.abs(den))
    gd = np.where(ok, np.real(num / np.where(ok, den, 1.0)), 0.0)
    return int(mround(np.mean(gd)))


def fftshift_index(P):
    """fftshift along a length-P vector: out[q] = X[(q - floor(P/2)) mod P]."""
    return (np.arange(P) - P // 2) % P


# ----------------------------------------------------------------------------- waveforms
def lfm_pulse(tau, fs, B, sign):
    """MTD/fun_MTD_produce.m:61-69: t = -tau/2 : ts : tau/2-ts;
    pulse = exp(j*2*pi*(f0*t + 0.5*K*t.^2)), f0 = 0, K = sign*B/tau."""
    ts = 1.0 / fs
    t = colon(-tau / 2.0, ts, tau / 2.0 - ts)
    K = sign * B / tau
    return np.exp(1j * 2.0 * np.pi * (0.5 * K * t * t))


def v2_params(P=332, R=3404, point_prt=None):
    """Radar parameters of MTD/main_produce_dataset_win_xzr_v2.m:22-45."""
    if point_prt is None:
        point_prt = [R, 228, 723, R - 951]
    p = dict(prtNum=P, fs=25e6, fc=9450e6, prt=232.76e-6, B=20e6,
             tao=[0.16e-6, 8e-6, 28e-6], point_prt=list(point_prt))
    p["prf"] = 1.0 / p["prt"]
    p["wavelength"] = C_LIGHT / p["fc"]
    p["deltaR"] = C_LIGHT / (2.0 * p["fs"])
    return p


def v2_pulses(params):
    """pulse1..3 of MTD/fun_MTD_produce.m:61-69 (pulse1 = sin(2*pi*t1+pi/2) is unused by PC)."""
    fs, B, tao = params["fs"], params["B"], params["tao"]
    ts = 1.0 / fs
    t1 = colon(-tao[0] / 2.0, ts, tao[0] / 2.0 - ts)
    pulse1 = np.sin(2.0 * np.pi * t1 + np.pi / 2.0)
    pulse2 = lfm_pulse(tao[1], fs, B, -1.0)   # K2 = -B/tao2  (:50)
    pulse3 = lfm_pulse(tao[2], fs, B, +1.0)   # K3 = +B/tao3  (:51)
    return pulse1, pulse2, pulse3


def mtd_zero_num(P, wavelength, prf, mtd_v=3.0, nd=None):
    """MTD_0_num = floor(MTD_V/deltaV), deltaV = lambda*prf/Nd/2
    (CFAR_WangCai/main_cfar.m:56-58; DMX_SignalProcessing_main_xzr.m:322-323,462)."""
    nd = P if nd is None else nd
    dv = wavelength * (prf / nd) / 2.0
    return int(np.floor(mtd_v / dv))


# ----------------------------------------------------------------------------- pulse compression
def fun_pulse_compression(s0, x):
    """MTD/fun_pulse_compression.m:10-39 (legacy :1-24): h = conj(fliplr(s0));
    N = len(h)+len(x)-1; y = ifft(fft(x,N).*fft(h,N)) -- MATLAB's exact FFT size."""
    h = np.conj(np.asarray(s0)[::-1])
    N = len(h) + len(x) - 1
    return np.fft.ifft(np.fft.fft(x, N) * np.fft.fft(h, N))


def fun_lss_pulse_compression(echo, pulse2, pulse3, p1, p2, p3, fir_shift=True,
                              offset2=None, offset3=None):
    """v2: MTD/fun_lss_pulse_compression.m:17-80 (fir_shift=True).
    legacy: MatlabProcess_xuzerui/fun_lss_pulse_compression.m:3-49 (fir_shift=False,
    offsets 75/160 = the lengths of the legacy pulses, :36-37).
    echo: P x R complex (rows = PRTs).  Returns P x R complex."""
    echo = np.asarray(echo, np.complex128)
    P, R = echo.shape
    sig1 = echo[:, :p1]                       # :23
    sig2 = echo[:, p1:p1 + p2]                # :24
    sig3 = echo[:, p1 + p2:R]                 # :25 (to the end of the row)
    out = np.zeros((P, R), np.complex128)     # :27
    b = FIR_TAPS_RAW / np.max(FIR_TAPS_RAW)   # :31-32
    off2 = len(pulse2) if offset2 is None else offset2   # :58
    off3 = len(pulse3) if offset3 is None else offset3   # :63
    delay1 = grpdelay_round_mean(b) if fir_shift else 0  # :47
    for i in range(P):                        # :36
        y1 = mfilter(b, sig1[i]) / 1.2        # :38-39
        if fir_shift:
            y1 = np.roll(y1, -delay1)         # circshift(y, -delay1)  :50
        out[i, :p1] = y1[:p1]                 # :51
        y2 = fun_pulse_compression(pulse2, sig2[i])    # :41
        y3 = fun_pulse_compression(pulse3, sig3[i])    # :42
        out[i, p1:p1 + p2] = y2[off2 - 1:off2 - 1 + p2]                   # :60
        out[i, p1 + p2:p1 + p2 + p3] = y3[off3 - 1:off3 - 1 + p3]         # :65
    return out


def dmx_matched_filter(ref, nfft, beta=4.5, normalize=True):
    """CFAR_WangCai/DMX_SignalProcessing_main_xzr.m:156-202:
    w2 = refData.'/norm(refData.'); H = conj(fft(w2.*kaiser(67,4.5).', FFT_num))."""
    w2 = np.asarray(ref, np.complex128).ravel()
    if normalize:
        w2 = w2 / np.linalg.norm(w2)                  # :165-167
    win = kaiser(len(w2), beta)                       # :185-187
    return np.conj(np.fft.fft(w2 * win, nfft))        # :202


def dmx_pulse_compression(echo, p_short, nfft, H, fir_short=True):
    """DMX_SignalProcessing_main_xzr.m:331-353: short = filter(b_raw,1,x(:,1:p_short));
    long = ifft(fft(x(:,p_short+1:end), nfft, 2) .* H, [], 2) (circular, nfft columns).
    Returns [short | long] side by side (the reference keeps them as two matrices)."""
    echo = np.asarray(echo, np.complex128)
    parts = []
    if p_short > 0:
        s = echo[:, :p_short]
        parts.append(mfilter(FIR_TAPS_RAW, s) if fir_short else s.copy())   # :343
    X = np.fft.fft(echo[:, p_short:], nfft, axis=1)                        # :348
    parts.append(np.fft.ifft(X * H[None, :], axis=1))                      # :352
    return np.concatenate(parts, axis=1)


# ----------------------------------------------------------------------------- MTD
def dmx_mtd_pair(pc_left, pc_right, nfft, m0):
    """DMX_SignalProcessing_main_xzr.m:414-426,462-465 (MTD_win_TYPE 1): per beam
    fft(pc .* hamming(prtNum), mtd_FFT_num, 1) -- no fftshift; sum = |L| + |R|,
    diff = |R| - |L|; rows [1:M0+1, mtd_FFT_num-M0+1:mtd_FFT_num] (1-based) of the sum zeroed."""
    pl = np.asarray(pc_left, np.complex128)
    pr = np.asarray(pc_right, np.complex128)
    w = hamming(pl.shape[0])[:, None]                                    # mtdWh (:211,227-228)
    ml = np.abs(np.fft.fft(pl * w, nfft, axis=0))                        # :416,418
    mr = np.abs(np.fft.fft(pr * w, nfft, axis=0))                        # :417,419
    s = ml + mr                                                          # :421-422
    d = mr - ml                                                          # :425-426
    zero = list(range(0, m0 + 1)) + list(range(nfft - m0, nfft))         # zeroSetFlagMTD (:463)
    s[zero, :] = 0.0                                                     # :464-465
    return s, d


def fun_Process_MTD(pc, window=None, nfft=None, shift=True):
    """MTD/fun_Process_MTD.m:13-40: for each range column,
    abs(fftshift(fft(col .* kaiser(P,8), P))).  The loop of :27-37 is kept."""
    pc = np.asarray(pc, np.complex128)
    P, R = pc.shape
    w = kaiser(P, 8.0) if window is None else np.asarray(window, np.float64)   # :17-18
    nd = P if nfft is None else nfft
    out = np.zeros((nd, R))
    for idx in range(R):                                   # :27
        sw = pc[:, idx] * w                                # :29
        f = np.fft.fft(sw, nd)                             # :31
        if shift:
            f = np.fft.fftshift(f)
        out[:, idx] = np.abs(f)                            # :33,36
    return out


def fun_0v_pressing(mtd, div=150):
    """MTD/fun_0v_pressing.m:13-24 (div 150) and CFAR_WangCai/fun_0v_pressing.m:2-7 (div 20):
    rows round(P/2)-round(P/div) : round(P/2)+round(P/div) (1-based) set to 0."""
    mtd = np.array(mtd, copy=True)
    P = mtd.shape[0]
    zv = int(mround(P / 2.0))
    k = int(mround(P / float(div)))
    mtd[zv - k - 1:zv + k, :] = 0.0
    return mtd


def zero_v_rows(P, div):
    """0-based [lo, hi) rows that fun_0v_pressing zeroes."""
    zv = int(mround(P / 2.0))
    k = int(mround(P / float(div)))
    return zv - k - 1, zv + k


def fun_MTD_produce_v2(echo, params, pulses=None, zero_v_div=150):
    """MTD/fun_MTD_produce.m:12-158: pulses (:61-69) -> fun_lss_pulse_compression (:86)
    -> fun_Process_MTD (:97-98) -> fun_0v_pressing (:102)."""
    _, pulse2, pulse3 = v2_pulses(params) if pulses is None else pulses
    pp = params["point_prt"]
    pc = fun_lss_pulse_compression(echo, pulse2, pulse3, pp[1], pp[2], pp[3], fir_shift=True)
    mtd = fun_Process_MTD(pc)
    if zero_v_div:
        mtd = fun_0v_pressing(mtd, zero_v_div)
    return mtd


def fun_lss_range_concate(prtNum, s):
    """MatlabProcess_xuzerui/fun_lss_range_concate.m:4-7, MATLAB's 1-based colons kept:
    concate_range = zeros(prtNum, 868);
    concate_range(:, 1:82)    = s(:, 1:82);
    concate_range(:, 83:318)  = s(:, 83+(82-75):325);
    concate_range(:, 319:868) = s(:, 325+(82+235-160):1031);"""
    s = np.asarray(s)
    out = np.zeros((prtNum, 868), s.dtype)
    out[:, 1 - 1:82] = s[:, 1 - 1:82]
    out[:, 83 - 1:318] = s[:, 83 + (82 - 75) - 1:325]
    out[:, 319 - 1:868] = s[:, 325 + (82 + 235 - 160) - 1:1031]
    return out


def fun_MTD_produce_legacy(echo, pulse2, pulse3, concat=False):
    """MatlabProcess_xuzerui/fun_MTD_produce.m:3-126 (hard-coded 82/242/707 segments,
    measured 75/160-sample pulses :54-60, no FIR circshift; its range concat at :70 is commented
    out).  concat=True: main.m's chain instead -- fun_lss_pulse_compression (:206),
    fun_lss_range_concate (:210-211), then the same MTD and 0-v."""
    pc = fun_lss_pulse_compression(echo, pulse2, pulse3, 82, 242, echo.shape[1] - 324,
                                   fir_shift=False, offset2=75, offset3=160)
    if concat:
        pc = fun_lss_range_concate(pc.shape[0], pc)
    return fun_0v_pressing(fun_Process_MTD(pc), 150)


def fun_MTD_produce_dmx_syn(echo, ref, zero_v_div=150):
    """Synthetic `dmx` preset: whole-row circular MF with
    refDDCDataMF1 (NFFT = R), then kaiser-8 / fftshift MTD and /150 0-v."""
    R = echo.shape[1]
    H = dmx_matched_filter(ref, R)
    pc = dmx_pulse_compression(echo, 0, R, H)
    mtd = fun_Process_MTD(pc)
    return fun_0v_pressing(mtd, zero_v_div) if zero_v_div else mtd


# ----------------------------------------------------------------------------- CFAR
def _windows(y, ncol, ref, save):
    """Reference-window bounds of Function_CFAR1D_sub.m:25-28 (1-based)."""
    return y - (save + ref), y - save - 1, y + save + 1, y + save + ref


def _side_means(D, cols_idx, y, ncol, ref, save):
    L1, L2, R1, R2 = _windows(y, ncol, ref, save)
    left_ok, right_ok = L1 >= 1, R2 <= ncol
    if not left_ok and not right_ok:
        raise CfarConfigError("CFAR window does not fit: %d cells < 2*(guard+ref)" % ncol)
    left = np.sum(D[:, L1 - 1:L2], axis=1) / float(ref) if left_ok else None
    right = np.sum(D[:, R1 - 1:R2], axis=1) / float(ref) if right_ok else None
    Lavg = left if left_ok else right        # :30-34
    Ravg = right if right_ok else left       # :35-39
    return Lavg, Ravg


def function_cfar1d_sub(D, ref, save, T, method, return_margin=False):
    """CFAR_WangCai/Function_CFAR1D_sub.m:1-75. Slides along the columns of D.
    flag(:,y) = D(:,y) >= T * (max|min)(meanL, meanR) with one-sided edge fallback."""
    D = np.asarray(D, np.float64)
    nrow, ncol = D.shape
    out = np.zeros((nrow, ncol))
    margin = np.full((nrow, ncol), np.inf)
    for y in range(1, ncol + 1):                                 # :17
        Lavg, Ravg = _side_means(D, None, y, ncol, ref, save)
        avg = np.maximum(Lavg, Ravg) if method == 0 else np.minimum(Lavg, Ravg)   # :40-44
        thr = avg * T                                            # :45
        out[:, y - 1] = (D[:, y - 1] >= thr).astype(np.float64)  # :46,68
        with np.errstate(divide="ignore", invalid="ignore"):
            margin[:, y - 1] = np.abs(D[:, y - 1] - thr) / np.abs(thr)
    return (out, margin) if return_margin else out


def function_cfar1d_sub_fixcells(D, ref, save, T, method, rows, cols, return_margin=False):
    """CFAR_WangCai/Function_CFAR1D_sub_fixCells.m:1-93: same window logic as
    Function_CFAR1D_sub but only at the given (1-based) rows/columns; others 0."""
    D = np.asarray(D, np.float64)
    nrow, ncol = D.shape
    out = np.zeros((nrow, ncol))
    margin = np.full((nrow, ncol), np.inf)
    rows0 = np.asarray(rows, int) - 1
    for y in cols:                                               # :23
        Lavg, Ravg = _side_means(D[rows0], None, y, ncol, ref, save)   # :34-48
        avg = np.maximum(Lavg, Ravg) if method == 0 else np.minimum(Lavg, Ravg)   # :50-54
        thr = avg * T
        out[rows0, y - 1] = (D[rows0, y - 1] >= thr).astype(np.float64)   # :58,85
        with np.errstate(divide="ignore", invalid="ignore"):
            margin[rows0, y - 1] = np.abs(D[rows0, y - 1] - thr) / np.abs(thr)
    return (out, margin) if return_margin else out


def executeCFAR(rdm, refR, saveR, TR, mR, refV, saveV, TV, mV, M0, rFlag, near_tol=None):
    """CFAR_WangCai/executeCFAR.m:1-93.  Returns (flag, flagV) as float 0/1 arrays.
    With near_tol, also returns an `ambiguous` mask of output cells whose value could
    flip under a relative perturbation of near_tol of the RDM (SURVEY.md §8d rule)."""
    rdm = np.asarray(rdm, np.float64)
    V, Rn = rdm.shape
    lo, hi = M0 + 1, V - M0                                      # rows M0+2 : V-M0  (:23)
    used = rdm[lo:hi, :]
    nv, nr = used.shape
    fv_used_T, mV_T = function_cfar1d_sub(used.T, refV, saveV, TV, mV, return_margin=True)  # :28
    fv_used, margV = fv_used_T.T, mV_T.T
    flagV = np.zeros((V, Rn))
    flagV[lo:hi, :] = fv_used                                    # :30-31
    amb_used = np.zeros((nv, nr), bool)
    if rFlag:                                                    # :35
        res = np.zeros((nv, nr))
        hits = np.argwhere(fv_used.T != 0)                       # find(): column-major order  :36
        for r0, v0 in hits:                                      # :45
            v, r = v0 + 1, r0 + 1                                # 1-based
            cells = [c for c in (r - 1, r, r + 1) if 1 <= c <= nr]   # :50-57
            row = used[v - 1:v, :]                               # :59
            det, marg = function_cfar1d_sub_fixcells(row, refR, saveR, TR, mR, [1], cells,
                                                     return_margin=True)   # :61
            nz = [c for c in cells if det[0, c - 1] != 0]        # find()  :64
            if nz:
                vals = [row[0, c - 1] for c in nz]
                best = nz[int(np.argmax(vals))]                  # first max  :68-70
                res[v - 1, best - 1] = 1.0                       # :78-84
            if near_tol is not None:
                amb = any(marg[0, c - 1] < near_tol for c in cells)
                if len(cells) > 1:
                    vals_all = np.array([row[0, c - 1] for c in cells])
                    srt = np.sort(vals_all)[::-1]
                    if srt[0] > 0 and (srt[0] - srt[1]) / srt[0] < near_tol:
                        amb = True
                if amb:
                    for c in cells:
                        amb_used[v - 1, c - 1] = True
        if near_tol is not None:
            # a Doppler decision that is near threshold can add or remove a hit at r,
            # which affects output cells r-1..r+1
            near_v = margV < near_tol
            for v0, r0 in np.argwhere(near_v):
                amb_used[v0, max(0, r0 - 1):min(nr, r0 + 2)] = True
        flag = np.zeros((V, Rn))
        flag[lo:hi, :] = res                                     # :89
    else:
        flag = flagV.copy()                                      # :91
        if near_tol is not None:
            amb_used = margV < near_tol
    if near_tol is None:
        return flag, flagV
    amb = np.zeros((V, Rn), bool)
    amb[lo:hi, :] = amb_used
    return flag, flagV, amb


def fun_CFARflag(mtd, refR, saveR, TR, mR, refV, saveV, TV, mV, M0, rFlag,
                 segments=((1, 82), (83, 318), (319, 868)), near_tol=None):
    """CFAR_WangCai/main_cfar.m:142-161 (a local function there): executeCFAR on each
    column segment (1-based inclusive bounds, default the hard-coded 1:82|83:318|319:868),
    reassembled into zeros(size(mtd)).  Returns (flag, flagV[, ambiguous])."""
    mtd = np.asarray(mtd, np.float64)
    flag = np.zeros(mtd.shape)
    flagV = np.zeros(mtd.shape)
    amb = np.zeros(mtd.shape, bool)
    for a, b in segments:
        r = executeCFAR(mtd[:, a - 1:b], refR, saveR, TR, mR, refV, saveV, TV, mV, M0, rFlag,
                        near_tol=near_tol)
        flag[:, a - 1:b] = r[0]
        flagV[:, a - 1:b] = r[1]
        if near_tol is not None:
            amb[:, a - 1:b] = r[2]
    return (flag, flagV, amb) if near_tol is not None else (flag, flagV)


def main_cfar_chain(mtd, cfar, segments, zero_v_div=20, near_tol=None):
    """CFAR_WangCai/main_cfar.m:88-93: abs -> fun_0v_pressing (the /20 copy when run
    from its folder) -> fun_CFARflag.  `cfar` = dict of executeCFAR's scalars."""
    m = np.abs(np.asarray(mtd, np.float64))
    if zero_v_div:
        m = fun_0v_pressing(m, zero_v_div)
    return fun_CFARflag(m, cfar["refR"], cfar["saveR"], cfar["TR"], cfar["methodR"],
                        cfar["refV"], cfar["saveV"], cfar["TV"], cfar["methodV"],
                        cfar["M0"], cfar["rFlag"], segments=segments, near_tol=near_tol)

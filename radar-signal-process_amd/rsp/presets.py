"""Parameter presets: the reference's `params` struct and CFAR scalars as engine specs.

Each preset restates how one MATLAB chain configures the hot path:
  v2      MTD/fun_MTD_produce.m:12-158 with the radar parameters of
          MTD/main_produce_dataset_win_xzr_v2.m:22-45 (3-segment PC: FIR with circshift,
          LFM matched filters of 200 / 700 samples; kaiser-8 MTD with fftshift; 0-v /150)
  legacy  MatlabProcess_xuzerui/fun_MTD_produce.m:3-126 (82/242/707 segments, measured
          75/160-sample pulses, no circshift)
  dmx     the synthetic DMX preset of SURVEY.md Appendix B: one circular matched filter over
          the whole row with refDDCDataMF1 x kaiser(67,4.5) / norm
          (CFAR_WangCai/DMX_SignalProcessing_main_xzr.m:156-202,348-352), NFFT = R
CFAR defaults follow CFAR_WangCai/main_cfar.m:40-58 (ref 5, guard 7, T 5, greatest-of,
range CFAR on, MTD_V = 3 m/s) and its /20 fun_0v_pressing (main_cfar.m:90-91).
"""
import ctypes as C
import math
import os
from dataclasses import dataclass, field

import numpy as np

from . import _capi as capi

C_LIGHT = 2.99792458e8
_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")

# MTD/fun_lss_pulse_compression.m:31 (same taps in the legacy and DMX code)
FIR_TAPS = np.array([-9, -7, -2, 10, 27, 40, 42, 24, -13, -57, -89, -86, -30, 77, 220, 364,
                     471, 511, 471, 364, 220, 77, -30, -86, -89, -57, -13, 24, 42, 40, 27, 10,
                     -2, -7, -9], dtype=np.float64)


def _mround(x):
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def _nextpow2(n):
    return 1 << max(6, int(math.ceil(math.log2(max(1, n)))))


def load_data(name):
    return np.load(os.path.join(_DATA, name + ".npy"), allow_pickle=False)


def kaiser(n, beta):
    if n == 1:
        return np.ones(1)
    k = np.arange(n, dtype=np.float64)
    r = (k - (n - 1) / 2.0) / ((n - 1) / 2.0)
    return np.i0(beta * np.sqrt(np.maximum(0.0, 1.0 - r * r))) / np.i0(beta)


def colon_len(a, d, b):
    q = (b - a) / d
    return (int(round(q)) if abs(q - round(q)) < 1e-9 * max(1.0, abs(q)) else int(math.floor(q))) + 1


def lfm(tau, fs, B, sign):
    """MTD/fun_MTD_produce.m:61-69: exp(j*2*pi*0.5*K*t.^2), t = -tau/2 : 1/fs : tau/2-1/fs."""
    ts = 1.0 / fs
    n = colon_len(-tau / 2.0, ts, tau / 2.0 - ts)
    t = -tau / 2.0 + ts * np.arange(n)
    return np.exp(1j * 2.0 * np.pi * (0.5 * (sign * B / tau) * t * t))


def radar_params(P=332, R=3404, point_prt=None, fs=25e6, fc=9450e6, prt=232.76e-6, B=20e6,
                 tao=(0.16e-6, 8e-6, 28e-6)):
    """The `params` struct of MTD/main_produce_dataset_win_xzr_v2.m:22-45."""
    if point_prt is None:
        point_prt = [R, 228, 723, R - 951]
    p = dict(prtNum=P, fs=fs, fc=fc, prt=prt, B=B, tao=list(tao), point_prt=list(point_prt))
    p["prf"] = 1.0 / prt
    p["wavelength"] = C_LIGHT / fc
    p["deltaR"] = C_LIGHT / (2.0 * fs)
    p["debug"] = dict(show_PC=0, show_FFT=0, graph=0)
    return p


@dataclass
class Segment:
    kind: int                      # capi.RSP_SEG_FIR / RSP_SEG_MF
    in_start: int
    in_len: int
    out_start: int
    out_len: int
    coef: np.ndarray               # FIR taps (real) / MF replica (complex)
    nfft: int = 0
    scale: float = 1.0
    fir_shift: int = 0


@dataclass
class Spec:
    """Everything rsp_create needs (rsp_params) plus the natural CFAR column segments."""
    name: str
    P: int
    R: int
    R_out: int
    segments: list
    window: int = capi.RSP_WIN_KAISER
    window_beta: float = 8.0
    fftshift: int = 1
    zero_v_div: int = 150
    cfar_segments: list = field(default_factory=list)   # 0-based [lo, hi)
    radar: dict = field(default_factory=dict)
    mtd_nfft: int = 0          # Doppler FFT length V (0 = P); DMX: 2048 over 1536 pulses
    beams: int = 1             # 2: DMX left/right pair, RDM = |X_L| + |X_R|
    zero_ends: int = 0         # DMX zeroSetFlagMTD: MTD_0_num + 1 (0 = fun_0v_pressing instead)
    # range concatenation between PC and MTD (fun_lss_range_concate, rsp_set_range_concat):
    # [(src_start, len), ...] of the pc_width PC columns; R_out is then their total
    concat: list = field(default_factory=list)
    pc_width: int = 0          # PC output columns (rsp_params.R_out); 0 = R_out

    @property
    def V(self):
        """Doppler rows of the RDM."""
        return self.mtd_nfft or self.P

    def to_c(self):
        """Build the ctypes rsp_params; returns (struct, keepalive list)."""
        prm = capi.rsp_params()
        prm.P, prm.R, prm.R_out = self.P, self.R, self.pc_width or self.R_out
        prm.nseg = len(self.segments)
        prm.window, prm.window_beta = self.window, self.window_beta
        prm.fftshift, prm.zero_v_div = self.fftshift, self.zero_v_div
        prm.mtd_nfft, prm.beams, prm.zero_ends = self.mtd_nfft, self.beams, self.zero_ends
        keep = []
        for i, s in enumerate(self.segments):
            g = prm.seg[i]
            g.kind, g.fir_shift = s.kind, s.fir_shift
            g.in_start, g.in_len, g.out_start, g.out_len = s.in_start, s.in_len, s.out_start, s.out_len
            g.nfft, g.scale = s.nfft, s.scale
            c = np.asarray(s.coef)
            re = np.ascontiguousarray(np.real(c), dtype=np.float64)
            im = np.ascontiguousarray(np.imag(c), dtype=np.float64)
            keep += [re, im]
            g.coef_len = c.size
            g.coef_re = re.ctypes.data_as(C.POINTER(C.c_double))
            g.coef_im = im.ctypes.data_as(C.POINTER(C.c_double))
        return prm, keep


def lss_spec(name, P, R, p1, p2, p3, pulse2, pulse3, fir_shift, radar=None):
    """3-segment pulse compression of fun_lss_pulse_compression (v2 :17-80, legacy :3-49)."""
    m3 = R - p1 - p2
    if m3 < 1 or p3 > m3:
        raise ValueError("segment 3 needs 1 <= p3 <= R - p1 - p2 (got R=%d p3=%d)" % (R, p3))
    segs = [
        Segment(capi.RSP_SEG_FIR, 0, p1, 0, p1, FIR_TAPS / FIR_TAPS.max(), scale=1.0 / 1.2,
                fir_shift=fir_shift),
        Segment(capi.RSP_SEG_MF, p1, p2, p1, p2, np.asarray(pulse2),
                nfft=_nextpow2(p2 + len(pulse2) - 1)),
        Segment(capi.RSP_SEG_MF, p1 + p2, m3, p1 + p2, p3, np.asarray(pulse3),
                nfft=_nextpow2(m3 + len(pulse3) - 1)),
    ]
    cfar_segs = [(0, p1), (p1, p1 + p2), (p1 + p2, R)]
    return Spec(name, P, R, R, segs, cfar_segments=cfar_segs, radar=radar or {})


def fir_group_delay(taps):
    """round(mean(grpdelay(b))) (MTD/fun_lss_pulse_compression.m:47): a symmetric
    (linear-phase) FIR has constant group delay (ntaps-1)/2."""
    taps = np.asarray(taps)
    if not np.allclose(taps, taps[::-1]):
        raise ValueError("non-symmetric FIR: group delay is not constant")
    return (len(taps) - 1) // 2


def v2(P=332, R=3404, point_prt=None, radar=None):
    """fun_MTD_produce v2 (MTD/fun_MTD_produce.m:12-158)."""
    rp = radar or radar_params(P, R, point_prt)
    pp = rp["point_prt"]
    pulse2 = lfm(rp["tao"][1], rp["fs"], rp["B"], -1.0)   # K2 = -B/tao2  (:50)
    pulse3 = lfm(rp["tao"][2], rp["fs"], rp["B"], +1.0)   # K3 = +B/tao3  (:51)
    return lss_spec("v2", P, R, pp[1], pp[2], pp[3], pulse2, pulse3,
                    fir_shift=fir_group_delay(FIR_TAPS), radar=rp)


# fun_lss_range_concate (MatlabProcess_xuzerui/fun_lss_range_concate.m:4-7): columns 1:82,
# 83+(82-75):325 and 325+(82+235-160):1031 (1-based) of the 1031 PC columns -> 868
LEGACY_CONCAT = [(0, 82), (89, 236), (481, 550)]


def legacy(P=1536, R=1031, concat=False):
    """MatlabProcess_xuzerui/fun_MTD_produce.m:3-126 (hard-coded 82/242/707, measured pulses,
    fc 5.5 GHz, PRT 64.88 us :24-38).  concat=True: main.m's chain, which concatenates the
    range segments between pulse compression and MTD (main.m:210-211, fun_lss_range_concate;
    commented out inside fun_MTD_produce.m:70): the MTD and CFAR then see 868 columns."""
    rp = dict(prtNum=P, fs=25e6, fc=5500e6, prt=64.88e-6, B=10e6,
              point_prt=[R, 82, 242, R - 324])
    rp["prf"] = 1.0 / rp["prt"]
    rp["wavelength"] = C_LIGHT / rp["fc"]
    spec = lss_spec("legacy", P, R, 82, 242, R - 324, load_data("legacy_pulse2"),
                    load_data("legacy_pulse3"), fir_shift=0, radar=rp)
    # fun_CFARflag's hard-coded split after fun_lss_range_concate (main_cfar.m:143-145)
    spec.cfar_segments = [(0, 82), (82, 318), (318, min(868, R))]
    if concat:
        if R != 1031:
            raise ValueError("fun_lss_range_concate indexes the 1031-column legacy row (got R=%d)" % R)
        spec.concat = list(LEGACY_CONCAT)
        spec.pc_width = R
        spec.R_out = sum(n for _, n in LEGACY_CONCAT)
        spec.name = "legacy_concat"
    return spec


def dmx_replica(name="refDDCDataMF1", beta=4.5):
    """w2 = refData.'/norm(refData) .* kaiser(67, 4.5).' (DMX_SignalProcessing_main_xzr.m:158-187)."""
    ref = load_data(name).astype(np.complex128)
    ref = ref / np.linalg.norm(ref)
    return ref * kaiser(len(ref), beta)


def dmx(P=128, R=4096, radar=None):
    """Synthetic DMX preset: whole-row circular matched filter, NFFT = R."""
    if R & (R - 1):
        raise ValueError("dmx preset needs a power-of-two R (NFFT = R)")
    rp = radar or radar_params(P, R)
    segs = [Segment(capi.RSP_SEG_MF, 0, R, 0, R, dmx_replica(), nfft=R)]
    return Spec("dmx", P, R, R, segs, cfar_segments=[(0, R)], radar=rp)


# DMX_SignalProcessing_main_xzr.m waveform 1 (:100-120): fs 12.5 MHz, PRT 52.08 us, 62 short +
# 504 long samples, FFT_num 512, mtd_FFT_num 2048, prtNum 1536; carrier from freValueGen.m
DMX_FS = 12.5e6
DMX_PRT = 52.08e-6
DMX_FC = 9365e6            # freValueGen(0 or 1)


def dmx_native(P=1536, R=566, point_short=62, fft_num=512, mtd_fft_num=2048, fc=DMX_FC, mtd_v=1.0):
    """The DMX chain at its native sizes (DMX_SignalProcessing_main_xzr.m:146,202,208-229,
    331-353,414-426,462-465): short part = filter(b_raw, 1, x) with the raw integer taps (no
    scale, no shift); long part = ifft(fft(x, 512) .* conj(fft(ref.*kaiser(67,4.5), 512)))
    (circular, 512 outputs); slow time = fft(pc .* hamming(P), 2048, 1) without fftshift for
    the left and right beams, RDM = |L| + |R|; rows 1:M0+1 and 2048-M0+1:2048 zeroed."""
    long_in = R - point_short
    if long_in > fft_num:
        raise ValueError("long part (%d) exceeds FFT_num %d" % (long_in, fft_num))
    R_out = point_short + fft_num
    segs = [Segment(capi.RSP_SEG_FIR, 0, point_short, 0, point_short, FIR_TAPS.astype(np.float64)),
            Segment(capi.RSP_SEG_MF, point_short, long_in, point_short, fft_num, dmx_replica(), nfft=fft_num)]
    prf = 1.0 / DMX_PRT
    wl = C_LIGHT / fc
    delta_v = wl * (prf / mtd_fft_num) / 2.0                      # :322-323
    m0 = int(math.floor(mtd_v / delta_v))                         # MTD_0_num (:462)
    rp = dict(prtNum=P, fs=DMX_FS, fc=fc, prt=DMX_PRT, prf=prf, wavelength=wl, mtd_v=mtd_v, M0=m0)
    return Spec("dmx_native", P, R, R_out, segs, window=capi.RSP_WIN_HAMMING, fftshift=0, zero_v_div=0,
                cfar_segments=[(0, point_short), (point_short, R_out)], radar=rp,
                mtd_nfft=mtd_fft_num, beams=2, zero_ends=m0 + 1)


def dmx_native_cfar(spec, T=7.0):
    """The DMX CFAR settings (:235-247): ref 5, guard 7, T 7, GO, range stage on; M0 =
    MTD_0_num; no /20 suppression (the zeroed rows are the stripped ones)."""
    return Cfar(TR=T, TV=T, M0=spec.radar["M0"], zero_v_div=0, segments=list(spec.cfar_segments))


PRESETS = {"v2": v2, "legacy": legacy, "legacy_concat": lambda P, R: legacy(P, R, concat=True), "dmx": dmx,
           "dmx_native": dmx_native}


def make(name, P, R):
    if name == "legacy":
        return legacy(P, R)
    if name == "legacy_concat":
        return legacy(P, R, concat=True)
    if name == "dmx_native":
        return dmx_native(P, R)
    return PRESETS[name](P, R)


def mtd_zero_num(P, wavelength, prf, mtd_v=3.0):
    """MTD_0_num = floor(MTD_V / (lambda * prf / P / 2)) (main_cfar.m:56-58)."""
    return int(math.floor(mtd_v / (wavelength * (prf / P) / 2.0)))


@dataclass
class Cfar:
    """The scalar arguments of executeCFAR (executeCFAR.m:1-2) + fun_CFARflag segmentation."""
    refR: int = 5
    saveR: int = 7
    TR: float = 5.0
    methodR: int = 0
    refV: int = 5
    saveV: int = 7
    TV: float = 5.0
    methodV: int = 0
    M0: int = 5
    rFlag: int = 1
    zero_v_div: int = 20
    segments: list = field(default_factory=list)   # 0-based [lo, hi); empty = whole row

    def to_c(self):
        c = capi.rsp_cfar_params()
        c.refR, c.saveR, c.methodR, c.TR = self.refR, self.saveR, self.methodR, self.TR
        c.refV, c.saveV, c.methodV, c.TV = self.refV, self.saveV, self.methodV, self.TV
        c.M0, c.rFlag, c.zero_v_div = self.M0, self.rFlag, self.zero_v_div
        c.nseg = len(self.segments)
        if c.nseg > capi.RSP_MAX_SEG:
            raise ValueError("at most %d CFAR segments" % capi.RSP_MAX_SEG)
        for i, (lo, hi) in enumerate(self.segments):
            c.seg_lo[i], c.seg_hi[i] = lo, hi
        return c

    def as_dict(self):
        return dict(refR=self.refR, saveR=self.saveR, TR=self.TR, methodR=self.methodR,
                    refV=self.refV, saveV=self.saveV, TV=self.TV, methodV=self.methodV,
                    M0=self.M0, rFlag=self.rFlag)


def default_cfar(spec, T=5.0, mtd_v=3.0, zero_v_div=20):
    if spec.name == "dmx_native":
        return dmx_native_cfar(spec)
    rp = spec.radar
    M0 = mtd_zero_num(spec.P, rp["wavelength"], rp["prf"], mtd_v)
    return Cfar(TR=T, TV=T, M0=M0, zero_v_div=zero_v_div, segments=list(spec.cfar_segments))

"""The DMX per-frame processing loop on the GPU (SURVEY.md rows a4/a8 + §8f-3): what
MatlabProcess_xuzerui/CFAR_WangCai/DMX_SignalProcessing_main_xzr.m does for one frame of the
two-beam long/short-pulse waveform (flag_Mode 1), from the left/right echo matrices to the
per-part target series:

  * scales (:93-96, :313-327): deltaR = c*ts/2, fc = freValueGen(freInd), rScale_short /
    rScale_long with the range calibration of :250-253, deltaV, fScale = fftshift(...), vScale;
  * pulse compression, 2048-point Doppler, |L|+|R| / |R|-|L|, zeroSetFlagMTD and executeCFAR on
    each part (:331-472): Engine(presets.dmx_native(fc=...)).run_dev -> sum, diff, flag, flagV;
  * motionParaMeasure on the short and the long part, for flag and for flagV (:489-516):
    Measure.measure_dev over the column windows of the same device planes.

Frames are batched ([batch][2 beams][P][R] complex64 on the device); everything between the
echo and the estimates stays in HBM.  The reference's own frame reader (frameDataRead_A) is
missing from the repository, so the echo matrices are the input here.
"""
import math

import numpy as np

from . import presets
from .engine import Engine
from .measure import Measure, angle_KvalueGen, freValueGen

# DMX_SignalProcessing_main_xzr.m:250-270
DMX_DEFAULTS = dict(rSysErr_short=0.0, rSysErr_long=62.0 * 12.0, rMeasureErr_short=297.0, rMeasureErr_long=92.0,
                    extraDots=2, rInterpTimes=8, vInterpTimes=4, eleAngleComp=0.0, eleAngleSysErr=0.0,
                    beamAngleStep=5.0, sysNum=1)


def dmx_scales(spec, freInd, **kw):
    """(rScale_short, rScale_long, vScale, deltaR, deltaV) of :93-96 and :313-327."""
    o = dict(DMX_DEFAULTS, **kw)
    fs, prf = spec.radar["fs"], spec.radar["prf"]
    deltaR = presets.C_LIGHT * (1.0 / fs) / 2.0
    lamda = presets.C_LIGHT / freValueGen(freInd)
    point_short = spec.cfar_segments[0][1]
    fft_num = spec.R_out - point_short
    N = spec.V
    rScale_short = np.arange(point_short) * deltaR + o["rSysErr_short"] - o["rMeasureErr_short"]
    rScale_long = np.arange(fft_num) * deltaR + o["rSysErr_long"] - o["rMeasureErr_long"]
    deltaDoppler = prf / N
    deltaV = lamda * deltaDoppler / 2.0
    fScale = np.fft.fftshift(np.arange(-N // 2, N // 2) * deltaDoppler)
    vScale = -lamda * fScale / 2.0
    return rScale_short, rScale_long, vScale, deltaR, deltaV


class DmxFrameProcessor:
    """One frequency number's DMX chain + measurement on one GPU."""

    def __init__(self, freInd=0, device=0, P=1536, R=566, **kw):
        self.o = dict(DMX_DEFAULTS, **kw)
        self.freInd = int(freInd)
        self.spec = presets.dmx_native(P=P, R=R, fc=freValueGen(self.freInd))
        self.cfar = presets.default_cfar(self.spec)
        self.eng = Engine(self.spec, device=device)
        self.meas = Measure(device)
        self.kValues = angle_KvalueGen(self.o["sysNum"])
        self.scales = dmx_scales(self.spec, self.freInd, **kw)
        self.device = self.meas.device

    def close(self):
        self.eng.close()
        self.meas.close()

    def process_dev(self, echo, beamPosNum, with_flagV=True, max_hits=4096):
        """echo: complex64 [batch][2][P][R] (left, right) on the device.  Returns a dict of
        device outputs: the planes (sum, diff, flag, flagV) and, per part ('short', 'long') and
        flag kind ('flag', 'flagV'), (est, cells, count) as Measure.measure_dev gives them."""
        import torch
        B = echo.shape[0]
        shp = (B, self.spec.V, self.spec.R_out)
        dev = self.device
        out = {k: torch.empty(shp, dtype=t, device=dev) for k, t in
               (("sum", torch.float32), ("diff", torch.float32), ("flag", torch.uint8), ("flagV", torch.uint8))}
        self.eng.run_dev(echo, rdm=out["sum"], diff=out["diff"], flag=out["flag"],
                         flagV=out["flagV"] if with_flagV else None, cfar=self.cfar)
        rS, rL, vS, dR, dV = self.scales
        o = self.o
        k_value = float(self.kValues[self.freInd, int(beamPosNum)])
        p = self.meas.params(o["extraDots"], dR, o["rInterpTimes"], dV, o["vInterpTimes"], k_value, beamPosNum,
                             o["beamAngleStep"], o["eleAngleComp"], o["eleAngleSysErr"], self.spec.radar["M0"])
        ps = self.spec.cfar_segments[0][1]
        for fk in ("flag", "flagV") if with_flagV else ("flag",):
            out[("short", fk)] = self.meas.measure_dev(out["sum"], out["diff"], out[fk], p, rS, vS,
                                                       max_hits=max_hits, cols=(0, ps))
            out[("long", fk)] = self.meas.measure_dev(out["sum"], out["diff"], out[fk], p, rL, vS,
                                                      max_hits=max_hits, cols=(ps, self.spec.R_out))
        return out

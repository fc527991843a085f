"""Post-detection measurement on the GPU: range, velocity and elevation of
every CFAR hit, with the reference's names and argument meaning:

  * motionParaMeasure(echo_MTD_sum, echo_MTD_diff, cfarResultFlag_Matrix, extraDots, rScale,
        deltaR, rInterpTimes, vScale, deltaV, vInterpTimes, kValues, beamPosNum,
        beamAngleStep, freInd, eleAngleComp, eleAngleSysErr, MTD_0_num)
        -> (rEstSeries, vEstSeries, eleAngleEstSeries)
    MatlabProcess_xuzerui/CFAR_WangCai/motionParaMeasure.m:1-88 (called at
    DMX_SignalProcessing_main_xzr.m:489-494), on the GPU through rsp_motion_measure_dev
    (csrc/rsp_measure.hip).  The matrices are V x R (MATLAB's orientation, which is also the
    device layout of rsp_pc_mtd_cfar_diff_dev's outputs); the series come back in MATLAB's
    find() order.  A hit the reference cannot re-anchor (it stops with an index error there)
    raises IndexError here too.
  * Measure.measure_dev(...): the batched device form, [batch][V][R] in (optionally a column
    window of wider planes), per-CPI hit lists out.
  * angle_KvalueGen(sysNum), freValueGen(freInd): the calibration lookups of
    CFAR_WangCai/angle_KvalueGen.m and freValueGen.m.

No CPU fallback: the estimates are computed only in librsp.so.
"""
import ctypes as C

import numpy as np

from . import _capi as capi

# angle_KvalueGen.m: one K-value row per frequency number (11 rows, freInd 0..10) and column
# per beam position (12).  The rows repeat in the pattern below (frequencies 0-2, 3-4, 5-6,
# 7-8, 9-10 share a row), so only the distinct rows are listed.
_K_ROW_OF_FREQ = (0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4)
_K_DISTINCT = {
    1: ((10.380672, 10.414385, 9.948529, 10.179451, 10.500966, 10.880367, 11.156690, 12.276938, 12.898726, 14.596353, 15.518284, 30.430223),
        (10.553918, 10.332526, 10.155857, 10.191538, 10.342200, 10.769444, 11.167994, 12.183270, 13.289346, 14.860170, 15.233340, 33.493266),
        (10.424651, 9.948311, 9.773556, 9.840688, 10.142961, 10.530585, 11.178810, 11.859324, 12.716404, 14.757746, 15.204941, 30.891074),
        (10.520613, 10.011845, 9.789657, 10.098063, 10.023637, 10.590518, 10.954758, 11.715884, 12.721137, 14.592968, 15.163915, 28.118921),
        (10.405303, 10.104511, 10.200153, 9.920508, 10.099613, 10.701100, 11.099405, 11.857029, 12.950606, 14.377440, 14.676968, 22.557463)),
    2: ((10.338870, 10.291381, 9.948466, 9.222804, 10.422373, 10.514297, 11.043671, 11.671526, 12.644140, 13.622801, 15.343592, 20.111603),
        (10.465372, 10.363734, 9.795664, 9.868073, 10.080984, 10.208166, 10.970078, 11.395584, 12.664564, 13.799594, 12.685487, 23.243726),
        (10.308061, 10.755928, 10.057556, 9.884201, 10.333652, 10.523828, 10.982471, 11.091260, 11.914261, 13.245791, 13.757134, 23.973037),
        (10.640704, 10.909189, 10.398377, 9.791719, 10.365195, 10.184979, 11.085054, 12.068282, 12.359290, 13.209102, 13.948980, 26.870156),
        (10.587029, 10.346590, 9.847715, 9.970153, 9.862467, 10.795310, 10.369297, 11.493181, 12.003133, 13.567793, 14.422600, 26.676481)),
}


def angle_KvalueGen(sysNum=1):  # noqa: N802 (reference name)
    """angle_KvalueGen.m: the 11 x 12 K-value table of radar `sysNum` (1 or 2); row freInd+1,
    column beamPosNum+1 (motionParaMeasure.m:79)."""
    if sysNum not in _K_DISTINCT:
        raise ValueError("angle_KvalueGen: no table for sysNum %r" % (sysNum,))
    rows = _K_DISTINCT[sysNum]
    return np.array([rows[i] for i in _K_ROW_OF_FREQ], dtype=np.float64)


def freValueGen(freInd):  # noqa: N802 (reference name)
    """freValueGen.m: carrier frequency [Hz] of frequency number 0..10 (0 and 1 share
    9365 MHz, then 10 MHz steps).  The reference leaves fc unset for other numbers, which is
    an error at its use; so is it here."""
    if freInd not in range(11):
        raise ValueError("freValueGen: frequency number %r outside 0..10" % (freInd,))
    return (9365.0 + 10.0 * max(freInd - 1, 0)) * 1e6


class Measure:
    """Owns an rsp context (the CFAR-only kind) for rsp_motion_measure_dev."""

    def __init__(self, device=0):
        import torch
        self.lib = capi.load_library()
        self.device = torch.device("cuda", device)
        ctx = C.c_void_p()
        capi.check(self.lib.rsp_create(C.byref(ctx), int(device), None), None)
        self.ctx = ctx

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.rsp_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def params(extraDots, deltaR, rInterpTimes, deltaV, vInterpTimes, k_value, beamPosNum, beamAngleStep,
               eleAngleComp, eleAngleSysErr, MTD_0_num):
        p = capi.rsp_measure_params()
        p.extra_dots, p.r_interp, p.v_interp = int(extraDots), int(rInterpTimes), int(vInterpTimes)
        p.mtd0_num, p.beam_pos_num = int(MTD_0_num), int(beamPosNum)
        p.delta_r, p.delta_v, p.k_value = float(deltaR), float(deltaV), float(k_value)
        p.beam_angle_step, p.ele_comp, p.ele_sys_err = float(beamAngleStep), float(eleAngleComp), float(eleAngleSysErr)
        return p

    def _dev(self, x, dtype):
        import torch
        if isinstance(x, torch.Tensor):
            return x.to(self.device, dtype).contiguous()
        return torch.as_tensor(np.ascontiguousarray(x), device=self.device).to(dtype).contiguous()

    def measure_dev(self, sum_rdm, diff_rdm, flag, params, r_scale, v_scale, max_hits=None, stream=None,
                    cols=None):
        """Batched: sum_rdm / diff_rdm float32 [batch][V][Rp], flag uint8 [batch][V][Rp] (device
        tensors, or arrays copied to the device).  cols = (lo, hi) measures the column window
        lo..hi-1 of every plane in place (e.g. DMX's short / long part), as the reference
        measures each part's own matrices; default all columns.  Returns (est float64
        [batch][max_hits][3], cells int32 [batch][max_hits][2] relative to the window, count
        int32 [batch][2]) on the device; count[:, 0] is the hit count of each CPI (hits past
        max_hits are counted, not written) and count[:, 1] the hits the reference would stop
        at with an index error."""
        import torch
        s = self._dev(sum_rdm, torch.float32)
        d = self._dev(diff_rdm, torch.float32)
        f = self._dev(flag, torch.uint8)
        if s.dim() == 2:
            s, d, f = s[None], d[None], f[None]
        B, V, Rp = s.shape
        if d.shape != s.shape or f.shape != s.shape:
            raise ValueError("measure_dev: sum %s, diff %s and flag %s differ in shape"
                             % (tuple(s.shape), tuple(d.shape), tuple(f.shape)))
        lo, hi = (0, Rp) if cols is None else (int(cols[0]), int(cols[1]))
        if not 0 <= lo < hi <= Rp:
            raise ValueError("measure_dev: column window %r outside 0..%d" % ((lo, hi), Rp))
        R = hi - lo
        rs = self._dev(np.asarray(r_scale, dtype=np.float64).reshape(-1), torch.float64)
        vs = self._dev(np.asarray(v_scale, dtype=np.float64).reshape(-1), torch.float64)
        if rs.numel() < R or vs.numel() < V:
            raise ValueError("measure_dev: rScale has %d of %d bins, vScale %d of %d rows" % (rs.numel(), R, vs.numel(), V))
        if max_hits is None:
            max_hits = min(V * R, 1 << 16)
        est = torch.empty((B, max_hits, 3), dtype=torch.float64, device=self.device)
        cells = torch.empty((B, max_hits, 2), dtype=torch.int32, device=self.device)
        count = torch.empty((B, 2), dtype=torch.int32, device=self.device)
        params.ld, params.cpi_stride = Rp, V * Rp
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        capi.check(self.lib.rsp_motion_measure_dev(
            self.ctx, s.data_ptr() + 4 * lo, d.data_ptr() + 4 * lo, f.data_ptr() + lo, V, R, B, C.byref(params),
            rs.data_ptr(), vs.data_ptr(), max_hits, est.data_ptr(), cells.data_ptr(), count.data_ptr(),
            C.c_void_p(st)), self.ctx)
        self._keep = (s, d, f, rs, vs)    # alive until the caller synchronises
        return est, cells, count

    @staticmethod
    def series(est, count, bad_raises=True):
        """Per-CPI (rEst, vEst, eleEst) numpy columns from measure_dev's outputs (synchronises)."""
        e, n = est.cpu().numpy(), count.cpu().numpy()
        out = []
        for b in range(e.shape[0]):
            if bad_raises and n[b, 1]:
                raise IndexError("motionParaMeasure: %d hit(s) too close to an edge for the reference's "
                                 "re-anchoring (motionParaMeasure.m:24-32, :51-59)" % n[b, 1])
            k = min(int(n[b, 0]), e.shape[1])
            out.append((e[b, :k, 0].copy(), e[b, :k, 1].copy(), e[b, :k, 2].copy()))
        return out

    def motionParaMeasure(self, echo_MTD_sum, echo_MTD_diff, cfarResultFlag_Matrix, extraDots, rScale, deltaR,  # noqa: N802
                          rInterpTimes, vScale, deltaV, vInterpTimes, kValues, beamPosNum, beamAngleStep, freInd,
                          eleAngleComp, eleAngleSysErr, MTD_0_num):
        """motionParaMeasure.m:1-88 for one V x R CPI; returns numpy column vectors."""
        import torch
        k_value = float(np.asarray(kValues)[int(freInd), int(beamPosNum)])          # kValues(freInd+1, beamPosNum+1)
        p = self.params(extraDots, deltaR, rInterpTimes, deltaV, vInterpTimes, k_value, beamPosNum, beamAngleStep,
                        eleAngleComp, eleAngleSysErr, MTD_0_num)
        V, R = tuple(np.shape(cfarResultFlag_Matrix)) if not isinstance(cfarResultFlag_Matrix, torch.Tensor) \
            else tuple(cfarResultFlag_Matrix.shape)
        flag = cfarResultFlag_Matrix
        if isinstance(flag, torch.Tensor):
            flag = (flag != 0).to(torch.uint8)
        else:
            flag = (np.asarray(flag) != 0).astype(np.uint8)
        est, cells, count = self.measure_dev(echo_MTD_sum, echo_MTD_diff, flag, p, rScale, vScale)
        n, bad = (int(x) for x in count[0].cpu())
        if n > est.shape[1]:
            est, cells, count = self.measure_dev(echo_MTD_sum, echo_MTD_diff, flag, p, rScale, vScale, max_hits=n)
        if bad:
            raise IndexError("motionParaMeasure: %d hit(s) too close to an edge for the reference's re-anchoring "
                             "(motionParaMeasure.m:24-32, :51-59)" % bad)
        e = est[0, :n].cpu().numpy()
        return e[:, 0].copy(), e[:, 1].copy(), e[:, 2].copy()

"""Echo pre-filters on the GPU, with the reference's names and meaning:

  * fun_iSTC(echo, stc_curve) -> (stc, eoch_iSTC)       MTD/fun_iSTC.m:2-17: the stc curve (dB
    per range bin, read with textread(..., '%f'); pass the file path or the values) zero-padded
    to the row length (:8-9), applied as echo(i,:) .* 10.^(stc/20) (:12-15).  A curve longer
    than the rows is a dimension error in MATLAB and a ValueError here.
  * fun_Process_MTI(ProSiganl, lag=30) -> MTI_Out        MTD/fun_Process_MTI.m:7-22: row m
    becomes x(m+30,:) - x(m,:) for m <= P-30, the last 30 rows stay zero (:9).  The mean it
    computes at :10-13 feeds only commented-out code and is not computed.
  * Prefilter.apply_dev(echo, out, gain, mti_lag): both on a [batch][P][R] complex64 device
    batch in one pass (rsp_prefilter_dev), e.g. ahead of Engine.run_dev.

No CPU fallback: the filters run only in librsp.so.
"""
import ctypes as C

import numpy as np

from . import _capi as capi


def read_stc_curve(stc_curve):
    """textread(path, '%f') or the values themselves, as a float64 vector."""
    if isinstance(stc_curve, (str, bytes)) or hasattr(stc_curve, "__fspath__"):
        with open(stc_curve, "r") as f:
            return np.array([float(t) for t in f.read().split()], dtype=np.float64)
    return np.asarray(stc_curve, dtype=np.float64).reshape(-1)


def istc_gain(stc_curve, R):
    """(stc, gain): stc zero-padded to R (fun_iSTC.m:8-9) and its linear gain 10^(stc/20) in
    fp64 (:14), as float32 for the kernel."""
    ini = read_stc_curve(stc_curve)
    if ini.size > R:
        raise ValueError("fun_iSTC: stc curve has %d values for %d range bins (MATLAB: dimension error)"
                         % (ini.size, R))
    stc = np.zeros(R, dtype=np.float64)
    stc[:ini.size] = ini
    return stc, (10.0 ** (stc / 20.0)).astype(np.float32)


class Prefilter:
    """Owns an rsp context (the CFAR-only kind) for rsp_prefilter_dev."""

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

    def _echo(self, x):
        import torch
        if isinstance(x, torch.Tensor):
            return x.to(self.device, torch.complex64).contiguous()
        return torch.as_tensor(np.ascontiguousarray(x, dtype=np.complex64), device=self.device)

    def apply_dev(self, echo, out=None, gain=None, mti_lag=0, stream=None):
        """echo complex64 [..., P, R] on the device -> out (same shape); gain float32 [R]
        (device tensor or array) or None; mti_lag 0 = no MTI.  Asynchronous on `stream`."""
        import torch
        x = self._echo(echo)
        P, R = x.shape[-2], x.shape[-1]
        batch = x.numel() // (P * R)
        if out is None:
            out = torch.empty_like(x)
        if out.shape != x.shape or out.dtype != torch.complex64 or not out.is_contiguous():
            raise ValueError("apply_dev: out must be a contiguous complex64 tensor of shape %s" % (tuple(x.shape),))
        g = None
        if gain is not None:
            g = gain if isinstance(gain, torch.Tensor) else torch.as_tensor(np.asarray(gain, np.float32))
            g = g.to(self.device, torch.float32).contiguous()
            if g.numel() != R:
                raise ValueError("apply_dev: %d gains for %d range bins" % (g.numel(), R))
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        capi.check(self.lib.rsp_prefilter_dev(self.ctx, x.data_ptr(), out.data_ptr(), P, R, batch,
                                              g.data_ptr() if g is not None else None, int(mti_lag),
                                              C.c_void_p(st)), self.ctx)
        self._keep = (x, g)   # alive until the caller synchronises
        return out

    def fun_iSTC(self, echo, stc_curve):  # noqa: N802 (reference name)
        """fun_iSTC.m:2-17 on a P x R echo (MATLAB orientation: rows = pulses); returns
        (stc, eoch_iSTC) with eoch_iSTC a device tensor."""
        x = self._echo(echo)
        stc, gain = istc_gain(stc_curve, x.shape[-1])
        return stc, self.apply_dev(x, gain=gain)

    def fun_Process_MTI(self, ProSiganl, lag=30):  # noqa: N802 (reference name)
        """fun_Process_MTI.m:7-22; returns MTI_Out as a device tensor."""
        return self.apply_dev(ProSiganl, mti_lag=lag)

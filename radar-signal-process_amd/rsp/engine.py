"""Engine: one rsp_ctx (one device, one parameter set) behind a Python object.

Host-buffer methods take/return numpy arrays and go through the synchronous C entry
points (the MEX path).  Device methods take torch tensors that already live on the GPU
and enqueue on the current torch stream (the benchmark path); torch is only used for
device memory and streams here -- all arithmetic happens in librsp's kernels.
"""
import ctypes as C

import numpy as np

from . import _capi as capi
from . import presets


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class Engine:
    def __init__(self, spec, device=0, chunk=0, streams=0):
        self.spec = spec          # None: CFAR-only context
        self.lib = capi.load_library()
        ctx = C.c_void_p()
        if spec is None:
            rc = self.lib.rsp_create(C.byref(ctx), int(device), None)
        else:
            prm, self._keep = spec.to_c()
            rc = self.lib.rsp_create(C.byref(ctx), int(device), C.byref(prm))
        capi.check(rc, None)
        self.ctx = ctx
        self.device = device
        if spec is not None and spec.concat:
            self.set_range_concat(spec.concat)
        if chunk:
            self.set_chunk(chunk)
        if streams:
            self.set_streams(streams)

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "ctx", None):
            self.lib.rsp_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_streams(self, n):
        """Chunk pipelines 1..4, or 0 for the library's mode-dependent default."""
        capi.check(self.lib.rsp_set_streams(self.ctx, int(n)), self.ctx)

    def set_range_concat(self, parts):
        """fun_lss_range_concate between PC and MTD: [(src_start, len), ...] of the PC columns
        (rsp_set_range_concat); [] restores the PC width.  The spec's R_out must match."""
        n = len(parts)
        src = (C.c_int64 * max(n, 1))(*[int(a) for a, _ in parts])
        ln = (C.c_int64 * max(n, 1))(*[int(b) for _, b in parts])
        capi.check(self.lib.rsp_set_range_concat(self.ctx, n, src, ln), self.ctx)

    def set_chunk(self, cpis):
        capi.check(self.lib.rsp_set_chunk(self.ctx, int(cpis)), self.ctx)

    def set_pc_split(self, enable):
        """Overlap-save blocks for matched filters longer than 4096 points (1, the default) or
        whole-length transforms (0) -- rsp_set_pc_split."""
        capi.check(self.lib.rsp_set_pc_split(self.ctx, int(enable)), self.ctx)

    def set_host_pipeline(self, cpis_per_chunk=0, copy_threads=0):
        """Host-buffer calls (pc_mtd_cfar / pc_mtd): CPIs per pipelined chunk and host copy
        threads (0 = the library defaults) -- rsp_set_host_pipeline."""
        capi.check(self.lib.rsp_set_host_pipeline(self.ctx, int(cpis_per_chunk), int(copy_threads)), self.ctx)

    def set_prefilter(self, gain=None, mti_lag=0):
        """Fuse iSTC (gain: [R] linear gains, e.g. rsp.prefilter.istc_gain) into pulse
        compression's echo load and MTI (lag, e.g. 30) into the MTD's load of the PC rows
        (rsp_set_prefilter); gain=None and mti_lag=0 switch them off."""
        g = None
        if gain is not None:
            g = np.ascontiguousarray(gain, dtype=np.float32)
            if g.shape != (self.spec.R,):
                raise ValueError("gain must have R = %d entries" % self.spec.R)
        ptr = g.ctypes.data_as(C.POINTER(C.c_float)) if g is not None else None
        capi.check(self.lib.rsp_set_prefilter(self.ctx, ptr, int(mti_lag)), self.ctx)

    @property
    def shape(self):
        """(Doppler rows, range bins) of one RDM."""
        return self.spec.V, self.spec.R_out

    # ------------------------------------------------------------------ host buffers
    @staticmethod
    def _echo_host(echo, layout):
        a = np.asarray(echo)
        if a.dtype == np.complex128:
            dt = capi.RSP_C128
        elif a.dtype == np.complex64:
            dt = capi.RSP_C64
        elif a.dtype == np.float16 and a.shape[-1] == 2:
            dt = capi.RSP_C32F16   # [..., 2] interleaved I/Q pairs
        else:
            a = a.astype(np.complex128)
            dt = capi.RSP_C128
        return np.ascontiguousarray(a), dt

    def _batch_dims(self, echo_shape, layout):
        P, R = self.spec.P, self.spec.R
        if layout == capi.RSP_COLMAJOR:
            # MATLAB P x R column-major arrives as numpy [..., R, P] C order
            tail = (R, P)
        else:
            tail = (P, R)
        if tuple(echo_shape[-2:]) != tail:
            raise ValueError("echo shape %s does not end in %s" % (echo_shape, tail))
        return int(np.prod(echo_shape[:-2])) if len(echo_shape) > 2 else 1

    def pc_mtd_cfar(self, echo, cfar=None, layout=capi.RSP_ROWMAJOR, out_layout=capi.RSP_ROWMAJOR,
                    want_flagV=True, out=None):
        """echo: [batch][P][R] complex (row-major) or MATLAB [batch][R][P] with layout=COLMAJOR.
        Returns rdm (float32) [, flag, flagV (uint8)] in out_layout; `out` = (rdm, flag, flagV)
        host arrays to fill instead of fresh ones (flag / flagV may be None)."""
        a, dt = self._echo_host(echo, layout)
        shape = a.shape if dt != capi.RSP_C32F16 else a.shape[:-1]
        batch = self._batch_dims(shape, layout)
        if batch % self.spec.beams:
            raise ValueError("a %d-beam context needs echo [batch, %d, P, R]" % (self.spec.beams, self.spec.beams))
        batch //= self.spec.beams
        P, Ro, V = self.spec.P, self.spec.R_out, self.spec.V
        oshape = (batch, V, Ro) if out_layout == capi.RSP_ROWMAJOR else (batch, Ro, V)
        rdm = np.empty(oshape, np.float32) if out is None else out[0]
        flag = flagV = None
        cp = None
        if cfar is not None:
            cp = cfar.to_c()
            if out is None:
                flag = np.empty(oshape, np.uint8)
                flagV = np.empty(oshape, np.uint8) if want_flagV else None
            else:
                flag, flagV = out[1], out[2]
        for o, want in ((rdm, np.float32), (flag, np.uint8), (flagV, np.uint8)):
            if o is not None and (o.shape != oshape or o.dtype != want or not o.flags.c_contiguous):
                raise ValueError("output arrays must be C-contiguous %s of shape %s" % (want.__name__, oshape))
        rc = self.lib.rsp_pc_mtd_cfar(self.ctx, _ptr(a), dt, layout, P, self.spec.R, batch,
                                      C.byref(cp) if cp is not None else None, _ptr(rdm), out_layout,
                                      _ptr(flag), _ptr(flagV))
        capi.check(rc, self.ctx)
        if cfar is None:
            return rdm
        return rdm, flag, flagV

    def pc_mtd(self, echo, layout=capi.RSP_ROWMAJOR, out_layout=capi.RSP_ROWMAJOR):
        return self.pc_mtd_cfar(echo, None, layout, out_layout)

    def cfar(self, rdm, cfar, layout=capi.RSP_ROWMAJOR):
        """rdm: [batch][V][R] float (or MATLAB [batch][R][V] with COLMAJOR).  -> flag, flagV."""
        r = np.ascontiguousarray(rdm, dtype=np.float32)
        if r.ndim == 2:
            r = r[None]
        batch = r.shape[0]
        V, R = (r.shape[1], r.shape[2]) if layout == capi.RSP_ROWMAJOR else (r.shape[2], r.shape[1])
        flag = np.empty(r.shape, np.uint8)
        flagV = np.empty(r.shape, np.uint8)
        cp = cfar.to_c()
        rc = self.lib.rsp_cfar(self.ctx, _ptr(r), layout, V, R, batch, C.byref(cp), _ptr(flag), _ptr(flagV))
        capi.check(rc, self.ctx)
        return flag, flagV

    # ------------------------------------------------------------------ device tensors
    @staticmethod
    def _stream_handle(stream):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        return C.c_void_p(s.cuda_stream)

    def run_dev(self, echo, rdm=None, flag=None, flagV=None, cfar=None, stream=None, diff=None):
        """echo: torch tensor [batch, P, R] complex64, or [batch, P, R, 2] float16 (I/Q); a
        two-beam context takes [batch, 2, P, R(, 2)] (beam 0 = left).  rdm [batch, V, R_out]
        float32, flag / flagV uint8 of the same shape (flagV optional); two beams: rdm is
        |L| + |R| and diff (optional) |R| - |L|.  Asynchronous on `stream` (default: torch's
        current stream)."""
        import torch
        if not echo.is_cuda or not echo.is_contiguous():
            raise ValueError("echo must be a contiguous CUDA tensor")
        nb = self.spec.beams
        lead = 1 if nb == 1 else 2
        if echo.dtype == torch.complex64:
            dt, batch = capi.RSP_C64, echo.shape[0]
            tail = tuple(echo.shape[1:])
        elif echo.dtype == torch.float16:
            dt, batch = capi.RSP_C32F16, echo.shape[0]
            tail = tuple(echo.shape[1:-1])
            if echo.shape[-1] != 2:
                raise ValueError("fp16 echo must be [..., P, R, 2]")
        else:
            raise ValueError("echo dtype must be complex64 or float16 I/Q")
        want_in = (self.spec.P, self.spec.R) if lead == 1 else (nb, self.spec.P, self.spec.R)
        if tail != want_in:
            raise ValueError("echo is %s, engine expects [batch, %s]" % (tuple(echo.shape), want_in))
        want = (batch, self.spec.V, self.spec.R_out)
        for t, dtp in ((rdm, torch.float32), (flag, torch.uint8), (flagV, torch.uint8), (diff, torch.float32)):
            if t is not None and (tuple(t.shape) != want or t.dtype != dtp or not t.is_contiguous() or not t.is_cuda):
                raise ValueError("output tensor must be contiguous CUDA %s of shape %s" % (dtp, want))
        if diff is not None and nb != 2:
            raise ValueError("diff output needs a two-beam context")
        cp = cfar.to_c() if cfar is not None else None
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None   # noqa: E731
        if nb == 2:
            rc = self.lib.rsp_pc_mtd_cfar_diff_dev(
                self.ctx, C.c_void_p(echo.data_ptr()), dt, batch, C.byref(cp) if cp is not None else None,
                ptr(rdm), ptr(diff), ptr(flag), ptr(flagV), self._stream_handle(stream))
        else:
            rc = self.lib.rsp_pc_mtd_cfar_dev(
                self.ctx, C.c_void_p(echo.data_ptr()), dt, batch, C.byref(cp) if cp is not None else None,
                ptr(rdm), ptr(flag), ptr(flagV), self._stream_handle(stream))
        capi.check(rc, self.ctx)

    def window_dev(self, frames, win, rdm=None, flag=None, flagV=None, cfar=None, stream=None):
        """Sliding-window stream (main_produce_dataset_win_xzr_v2.m:94-144).
        frames: [beams, F+1, P, R] complex64 (or [..., 2] float16 I/Q) consecutive frames;
        outputs [beams, F, win, P, R_out] -- window i of frame pair (n, n+1) is rows
        [round(i*P/win), +P) of [frame n; frame n+1]."""
        import torch
        if not frames.is_cuda or not frames.is_contiguous():
            raise ValueError("frames must be a contiguous CUDA tensor")
        if frames.dtype == torch.complex64:
            dt, lead = capi.RSP_C64, tuple(frames.shape[:2])
            tail = tuple(frames.shape[2:])
        elif frames.dtype == torch.float16 and frames.shape[-1] == 2:
            dt, lead = capi.RSP_C32F16, tuple(frames.shape[:2])
            tail = tuple(frames.shape[2:4])
        else:
            raise ValueError("frames must be complex64 [beams, F+1, P, R] or float16 [beams, F+1, P, R, 2]")
        if len(lead) != 2 or tail != (self.spec.P, self.spec.R) or lead[1] < 2:
            raise ValueError("frames is %s, engine expects [beams, F+1>=2, %d, %d]"
                             % (tuple(frames.shape), self.spec.P, self.spec.R))
        beams, nf = lead[0], lead[1] - 1
        want = (beams, nf, int(win), self.spec.P, self.spec.R_out)
        for t, dtp in ((rdm, torch.float32), (flag, torch.uint8), (flagV, torch.uint8)):
            if t is not None and (tuple(t.shape) != want or t.dtype != dtp or not t.is_contiguous() or not t.is_cuda):
                raise ValueError("output tensor must be contiguous CUDA %s of shape %s" % (dtp, want))
        cp = cfar.to_c() if cfar is not None else None
        rc = self.lib.rsp_window_pc_mtd_cfar_dev(
            self.ctx, C.c_void_p(frames.data_ptr()), dt, beams, nf, int(win), C.byref(cp) if cp is not None else None,
            C.c_void_p(rdm.data_ptr()) if rdm is not None else None,
            C.c_void_p(flag.data_ptr()) if flag is not None else None,
            C.c_void_p(flagV.data_ptr()) if flagV is not None else None,
            self._stream_handle(stream))
        capi.check(rc, self.ctx)

    def mtd_dev(self, pc, rdm=None, flag=None, flagV=None, cfar=None, stream=None):
        """MTD + 0-v (+ CFAR) on pulse-compressed rows pc [batch, (beams,) P, R_out] complex64
        (e.g. from pc_dev); outputs as run_dev."""
        import torch
        if not pc.is_cuda or not pc.is_contiguous() or pc.dtype != torch.complex64:
            raise ValueError("pc must be a contiguous CUDA complex64 tensor")
        batch = pc.shape[0]
        want_in = (self.spec.P, self.spec.R_out) if self.spec.beams == 1 else (self.spec.beams, self.spec.P,
                                                                              self.spec.R_out)
        if tuple(pc.shape[1:]) != want_in:
            raise ValueError("pc is %s, engine expects [batch, %s]" % (tuple(pc.shape), want_in))
        want = (batch, self.spec.V, self.spec.R_out)
        for t, dtp in ((rdm, torch.float32), (flag, torch.uint8), (flagV, torch.uint8)):
            if t is not None and (tuple(t.shape) != want or t.dtype != dtp or not t.is_contiguous() or not t.is_cuda):
                raise ValueError("output tensor must be contiguous CUDA %s of shape %s" % (dtp, want))
        cp = cfar.to_c() if cfar is not None else None
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None   # noqa: E731
        rc = self.lib.rsp_mtd_cfar_dev(self.ctx, C.c_void_p(pc.data_ptr()), batch,
                                       C.byref(cp) if cp is not None else None, ptr(rdm), ptr(flag), ptr(flagV),
                                       self._stream_handle(stream))
        capi.check(rc, self.ctx)

    def pc_dev(self, echo, out, stream=None):
        """Pulse compression alone: out [batch, P, R_out] complex64."""
        import torch
        dt = capi.RSP_C64 if echo.dtype == torch.complex64 else capi.RSP_C32F16
        rc = self.lib.rsp_pc_dev(self.ctx, C.c_void_p(echo.data_ptr()), dt, echo.shape[0],
                                 C.c_void_p(out.data_ptr()), self._stream_handle(stream))
        capi.check(rc, self.ctx)

    def profile(self, enable=True, every=1):
        """Start (and reset) or stop per-kernel HIP-event timing inside librsp; `every` = N
        brackets every N-th launch only (sampled timing inside a throughput measurement)."""
        capi.check(self.lib.rsp_profile(self.ctx, int(every) if enable else 0), self.ctx)

    def profile_read(self):
        """{kernel name: (total ms, launches)} since profile(True)."""
        ms = (C.c_double * capi.RSP_NKERNELS)()
        n = (C.c_int64 * capi.RSP_NKERNELS)()
        capi.check(self.lib.rsp_profile_read_n(self.ctx, ms, n, capi.RSP_NKERNELS), self.ctx)
        return {capi.KERNEL_NAMES[k]: (ms[k], n[k]) for k in range(capi.RSP_NKERNELS) if n[k]}

    def cfar_dev(self, rdm, flag, flagV=None, cfar=None, stream=None):
        b, V, R = rdm.shape
        cp = cfar.to_c()
        rc = self.lib.rsp_cfar_dev(self.ctx, C.c_void_p(rdm.data_ptr()), V, R, b, C.byref(cp),
                                   C.c_void_p(flag.data_ptr()),
                                   C.c_void_p(flagV.data_ptr()) if flagV is not None else None,
                                   self._stream_handle(stream))
        capi.check(rc, self.ctx)


def engine_for(name, P, R, device=0, chunk=0):
    return Engine(presets.make(name, P, R), device=device, chunk=chunk)

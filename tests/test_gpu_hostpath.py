"""The pipelined host-buffer path (rsp_pc_mtd_cfar / rsp_pc_mtd with pageable host arrays, the
MEX drop-in for MTD/main_produce_dataset_win_xzr_v2.m:136's one-CPI fun_MTD_produce calls):
chunked H2D / chain / D2H through pinned staging rings must give exactly the device path's
outputs -- whatever the chunking, the copy-thread count, the input dtype and the layouts
(integer/layout work: bit-exact)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _engine(P, R):
    from rsp import presets
    from rsp.engine import Engine
    return Engine(presets.v2(P, R), device=0)


def _dev(torch, eng, echo64, cf):
    """The device path on the same (complex64) samples: rdm, flag, flagV row-major."""
    B = echo64.shape[0]
    V, Ro = eng.shape
    d = torch.from_numpy(echo64).cuda()
    rdm = torch.empty((B, V, Ro), dtype=torch.float32, device="cuda")
    flag = torch.empty((B, V, Ro), dtype=torch.uint8, device="cuda")
    fv = torch.empty((B, V, Ro), dtype=torch.uint8, device="cuda")
    eng.run_dev(d, rdm=rdm, flag=flag, flagV=fv, cfar=cf)
    torch.cuda.synchronize()
    return rdm.cpu().numpy(), flag.cpu().numpy(), fv.cpu().numpy()


@pytest.mark.parametrize("P,R,batch,chunk,threads", [
    (64, 1024, 7, 3, 0),      # 3 chunks, the last one short
    (64, 1024, 1, 0, 0),      # MATLAB's granularity: one CPI per call
    (64, 1024, 9, 1, 1),      # one CPI per chunk, one copy thread
    (128, 4096, 11, 0, 0),    # by size: 32 MiB of C128 input = 4 CPIs per chunk, 3 chunks
    (128, 4096, 1, 0, 5),     # one 8 MiB CPI: one pinned piece per direction plane
])
def test_host_path_equals_device_path(torch_cuda, P, R, batch, chunk, threads):
    from rsp import _capi as capi
    from rsp import presets, synth
    eng = _engine(P, R)
    cf = presets.default_cfar(eng.spec)
    echo = synth.echo_numpy(eng.spec, batch, seed=77 + batch).astype(np.complex64)
    want = _dev(torch_cuda, eng, echo, cf)
    eng.set_host_pipeline(chunk, threads)
    # MATLAB layout: complex double, column-major in and out
    col = np.ascontiguousarray(np.swapaxes(echo.astype(np.complex128), 1, 2))
    got = eng.pc_mtd_cfar(col, cf, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR)
    for g, w in zip(got, want):
        assert np.array_equal(np.swapaxes(g, 1, 2), w)
    # row-major complex64 in and out, without flagV
    rdm, flag, fv = eng.pc_mtd_cfar(echo, cf, want_flagV=False)
    assert fv is None and np.array_equal(rdm, want[0]) and np.array_equal(flag, want[1])
    # PC + MTD only
    assert np.array_equal(eng.pc_mtd(echo), want[0])
    eng.close()


def test_host_path_repeated_calls_and_fp16(torch_cuda):
    """Back-to-back calls reuse the rings and slots (events from the previous call) and the
    fp16 I/Q input goes through the same pipeline."""
    torch = torch_cuda
    from rsp import presets, synth
    eng = _engine(64, 2048)
    cf = presets.default_cfar(eng.spec)
    eng.set_host_pipeline(2, 0)
    for seed in (1, 2, 3):
        echo = synth.echo_numpy(eng.spec, 5, seed=seed).astype(np.complex64)
        want = _dev(torch, eng, echo, cf)
        got = eng.pc_mtd_cfar(echo, cf)
        for g, w in zip(got, want):
            assert np.array_equal(g, w)
    echo = synth.echo_numpy(eng.spec, 3, seed=9).astype(np.complex64)
    iq = np.ascontiguousarray(np.stack([echo.real, echo.imag], axis=-1).astype(np.float16))   # [3, P, R, 2]
    V, Ro = eng.shape
    rdm = torch.empty((3, V, Ro), dtype=torch.float32, device="cuda")
    flag = torch.empty((3, V, Ro), dtype=torch.uint8, device="cuda")
    eng.run_dev(torch.from_numpy(iq).cuda(), rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    got = eng.pc_mtd_cfar(iq, cf, want_flagV=False)
    assert np.array_equal(got[0], rdm.cpu().numpy()) and np.array_equal(got[1], flag.cpu().numpy())
    eng.close()


@pytest.mark.parametrize("chunk", [1, 2])
def test_host_path_two_beam_dmx(torch_cuda, chunk):
    """A two-beam (DMX) context through the host pipeline: in_cpi / dev_cpi scale by the beams
    and the column-major ingest converts batch * beams planes.  MATLAB's layout (C128, P x R
    column-major per beam), chunks smaller than the batch: bit-exact against the device path on
    the same complex64 samples."""
    torch = torch_cuda
    from rsp import _capi as capi
    from rsp import presets
    from rsp.engine import Engine
    spec = presets.dmx_native()
    eng = Engine(spec, device=0)
    cf = presets.dmx_native_cfar(spec)
    B = 3
    rng = np.random.default_rng(4040 + chunk)
    e = ((rng.standard_normal((B, 2, spec.P, spec.R)) + 1j * rng.standard_normal((B, 2, spec.P, spec.R)))
         * np.sqrt(0.5)).astype(np.complex64)
    V, Ro = eng.shape
    rdm = torch.empty((B, V, Ro), dtype=torch.float32, device="cuda")
    flag = torch.empty((B, V, Ro), dtype=torch.uint8, device="cuda")
    fv = torch.empty((B, V, Ro), dtype=torch.uint8, device="cuda")
    eng.run_dev(torch.from_numpy(e).cuda(), rdm=rdm, flag=flag, flagV=fv, cfar=cf)
    torch.cuda.synchronize()
    want = (rdm.cpu().numpy(), flag.cpu().numpy(), fv.cpu().numpy())
    eng.set_host_pipeline(chunk, 0)
    col = np.ascontiguousarray(np.swapaxes(e.astype(np.complex128), 2, 3))   # [B, beams, R, P]
    got = eng.pc_mtd_cfar(col, cf, layout=capi.RSP_COLMAJOR)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    rdm2, flag2, _ = eng.pc_mtd_cfar(e, cf, want_flagV=False)   # row-major complex64
    assert np.array_equal(rdm2, want[0]) and np.array_equal(flag2, want[1])
    eng.close()


def test_f64_entry_points_equal_float_forms(torch_cuda):
    """rsp_pc_mtd_cfar_f64 / rsp_cfar_f64 (MATLAB's double outputs and input, widened / narrowed
    on the copy threads piece by piece): the same values as the float / byte forms, exactly, for
    one CPI per call (the MEX granularity) and a chunked batch, in both layouts."""
    import ctypes as C
    from rsp import _capi as capi
    from rsp import presets, synth
    eng = _engine(128, 4096)
    cf = presets.default_cfar(eng.spec)
    cp = cf.to_c()
    lib = eng.lib
    V, Ro = eng.shape
    P, R = eng.spec.P, eng.spec.R
    ptr = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None   # noqa: E731
    for B, chunk, lay in ((1, 0, capi.RSP_COLMAJOR), (5, 2, capi.RSP_ROWMAJOR)):
        eng.set_host_pipeline(chunk, 0)
        echo = synth.echo_numpy(eng.spec, B, seed=900 + B).astype(np.complex128)
        if lay == capi.RSP_COLMAJOR:
            echo = np.ascontiguousarray(np.swapaxes(echo, 1, 2))
        oshape = (B, V, Ro) if lay == capi.RSP_ROWMAJOR else (B, Ro, V)
        r32, f8, v8 = np.empty(oshape, np.float32), np.empty(oshape, np.uint8), np.empty(oshape, np.uint8)
        assert lib.rsp_pc_mtd_cfar(eng.ctx, ptr(echo), capi.RSP_C128, lay, P, R, B, C.byref(cp), ptr(r32), lay,
                                   ptr(f8), ptr(v8)) == 0
        r64, f64, v64 = (np.full(oshape, np.nan), np.full(oshape, 7.0), np.full(oshape, 7.0))
        assert lib.rsp_pc_mtd_cfar_f64(eng.ctx, ptr(echo), capi.RSP_C128, lay, P, R, B, C.byref(cp), ptr(r64), lay,
                                       ptr(f64), ptr(v64)) == 0
        assert np.array_equal(r64, r32.astype(np.float64))
        assert np.array_equal(f64, f8.astype(np.float64)) and np.array_equal(v64, v8.astype(np.float64))
        # RDM only (fun_MTD_produce)
        r64b = np.full(oshape, np.nan)
        assert lib.rsp_pc_mtd_cfar_f64(eng.ctx, ptr(echo), capi.RSP_C128, lay, P, R, B, None, ptr(r64b), lay,
                                       None, None) == 0
        assert np.array_equal(r64b, r64)
        # executeCFAR on that RDM, double in / out, against the float form
        rin = r64.astype(np.float64)
        cf8, cv8 = np.empty(oshape, np.uint8), np.empty(oshape, np.uint8)
        assert lib.rsp_cfar(eng.ctx, ptr(np.ascontiguousarray(rin.astype(np.float32))), lay, V, Ro, B, C.byref(cp),
                            ptr(cf8), ptr(cv8)) == 0
        cf64, cv64 = np.full(oshape, 7.0), np.full(oshape, 7.0)
        assert lib.rsp_cfar_f64(eng.ctx, ptr(rin), lay, V, Ro, B, C.byref(cp), ptr(cf64), ptr(cv64)) == 0
        assert np.array_equal(cf64, cf8.astype(np.float64)) and np.array_equal(cv64, cv8.astype(np.float64))
        assert cf64.sum() > 0
    eng.close()


@pytest.mark.parametrize("P,R,batch", [(64, 1024, 1), (64, 1024, 6), (128, 4096, 1), (128, 4096, 3)])
def test_one_chunk_calls_stage_through_pinned_memory(torch_cuda, P, R, batch):
    """A call whose batch fits one chunk (the MEX granularity) runs the one-chunk path: the
    ingest transposes / copies read the echo from pinned staging piece by piece, and the output
    transposes / copies write pinned staging part by part while the copy threads deliver earlier
    parts.  Back-to-back calls with new inputs (the staging is reused: no stale lines), both
    layouts, C128 / C64 / fp16 inputs, with and without flagV and CFAR, and the double outputs:
    all bit-exact against the device path."""
    torch = torch_cuda
    import ctypes as C
    from rsp import _capi as capi
    from rsp import presets, synth
    eng = _engine(P, R)
    cf = presets.default_cfar(eng.spec)
    eng.set_host_pipeline(0, 0)
    V, Ro = eng.shape
    for seed in (11, 12, 13):
        echo = synth.echo_numpy(eng.spec, batch, seed=seed * 10 + batch).astype(np.complex64)
        want = _dev(torch, eng, echo, cf)
        col = np.ascontiguousarray(np.swapaxes(echo.astype(np.complex128), 1, 2))
        got = eng.pc_mtd_cfar(col, cf, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR)
        for g, w in zip(got, want):
            assert np.array_equal(np.swapaxes(g, 1, 2), w)
        got = eng.pc_mtd_cfar(echo, cf)   # row-major C64 in and out
        for g, w in zip(got, want):
            assert np.array_equal(g, w)
        rdm, flag, fv = eng.pc_mtd_cfar(col, cf, layout=capi.RSP_COLMAJOR, want_flagV=False)
        assert fv is None and np.array_equal(rdm, want[0]) and np.array_equal(flag, want[1])
        assert np.array_equal(eng.pc_mtd(echo), want[0])
    # MATLAB's double outputs (the fun_MTD_produce shim's call), column-major
    lib = eng.lib
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)   # noqa: E731
    r64 = np.full((batch, Ro, V), np.nan)
    assert lib.rsp_pc_mtd_cfar_f64(eng.ctx, ptr(col), capi.RSP_C128, capi.RSP_COLMAJOR, P, R, batch, None, ptr(r64),
                                   capi.RSP_COLMAJOR, None, None) == 0
    assert np.array_equal(np.swapaxes(r64, 1, 2), want[0].astype(np.float64))
    # fp16 I/Q, column-major ([b][R][P] of half2) and row-major
    iq = np.stack([echo.real, echo.imag], axis=-1).astype(np.float16)   # [b, P, R, 2]
    rdm = torch.empty((batch, V, Ro), dtype=torch.float32, device="cuda")
    flag = torch.empty((batch, V, Ro), dtype=torch.uint8, device="cuda")
    eng.run_dev(torch.from_numpy(np.ascontiguousarray(iq)).cuda(), rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    w16 = (rdm.cpu().numpy(), flag.cpu().numpy())
    got = eng.pc_mtd_cfar(np.ascontiguousarray(iq), cf, want_flagV=False)
    assert np.array_equal(got[0], w16[0]) and np.array_equal(got[1], w16[1])
    iqc = np.ascontiguousarray(np.swapaxes(iq, 1, 2))                    # [b, R, P, 2]
    got = eng.pc_mtd_cfar(iqc, cf, layout=capi.RSP_COLMAJOR, want_flagV=False)
    assert np.array_equal(got[0], w16[0]) and np.array_equal(got[1], w16[1])
    eng.close()


def test_one_chunk_two_beam(torch_cuda):
    """The one-chunk path with a two-beam (DMX) context: batch * beams input planes."""
    torch = torch_cuda
    from rsp import _capi as capi
    from rsp import presets
    from rsp.engine import Engine
    spec = presets.dmx_native()
    eng = Engine(spec, device=0)
    cf = presets.dmx_native_cfar(spec)
    eng.set_host_pipeline(0, 0)
    B = 1
    rng = np.random.default_rng(5151)
    e = ((rng.standard_normal((B, 2, spec.P, spec.R)) + 1j * rng.standard_normal((B, 2, spec.P, spec.R)))
         * np.sqrt(0.5)).astype(np.complex64)
    V, Ro = eng.shape
    rdm = torch.empty((B, V, Ro), dtype=torch.float32, device="cuda")
    flag = torch.empty((B, V, Ro), dtype=torch.uint8, device="cuda")
    fv = torch.empty((B, V, Ro), dtype=torch.uint8, device="cuda")
    eng.run_dev(torch.from_numpy(e).cuda(), rdm=rdm, flag=flag, flagV=fv, cfar=cf)
    torch.cuda.synchronize()
    want = (rdm.cpu().numpy(), flag.cpu().numpy(), fv.cpu().numpy())
    col = np.ascontiguousarray(np.swapaxes(e.astype(np.complex128), 2, 3))
    got = eng.pc_mtd_cfar(col, cf, layout=capi.RSP_COLMAJOR)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    rdm2, flag2, _ = eng.pc_mtd_cfar(e, cf, want_flagV=False)
    assert np.array_equal(rdm2, want[0]) and np.array_equal(flag2, want[1])
    eng.close()


def test_cfar_f64_dma_fallback_matches_cfar(torch_cuda):
    """rsp_cfar_f64 beyond the one-chunk limit (more than kParts = 16 output parts: batch 20 with
    flagV) takes the DMA pipeline instead of pinned staging: the double RDM narrowed by the copy
    threads on its way into the pinned input ring (h2d_pieces narrow 2), the u8 flag transposes for
    MATLAB's layout, and the flags widened to double as their pieces land (d2h widen 2).  Both
    layouts, bit-exact against rsp_cfar on the same (float-representable) values."""
    import ctypes as C
    from rsp import _capi as capi
    from rsp import presets
    from rsp.engine import Engine
    eng = Engine(presets.v2(64, 1024))
    cf = presets.default_cfar(eng.spec)
    cp = cf.to_c()
    lib = eng.lib
    V, R, B = 64, 1024, 20
    rng = np.random.default_rng(77)
    rdm = np.abs(rng.standard_normal((B, V, R)) + 1j * rng.standard_normal((B, V, R))).astype(np.float32)
    rdm[:, 20, 300] = 60.0
    rdm[:, 45, 700:703] = [30.0, 40.0, 35.0]
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)   # noqa: E731
    for lay in (capi.RSP_ROWMAJOR, capi.RSP_COLMAJOR):
        x = rdm if lay == capi.RSP_ROWMAJOR else np.ascontiguousarray(np.swapaxes(rdm, 1, 2))
        f8, v8 = np.empty(x.shape, np.uint8), np.empty(x.shape, np.uint8)
        assert lib.rsp_cfar(eng.ctx, ptr(x), lay, V, R, B, C.byref(cp), ptr(f8), ptr(v8)) == 0
        x64 = x.astype(np.float64)
        f64, v64 = np.full(x.shape, 7.0), np.full(x.shape, 7.0)
        assert lib.rsp_cfar_f64(eng.ctx, ptr(x64), lay, V, R, B, C.byref(cp), ptr(f64), ptr(v64)) == 0
        assert np.array_equal(f64, f8.astype(np.float64)) and np.array_equal(v64, v8.astype(np.float64))
        assert v8.sum() > 0
    eng.close()


@pytest.mark.parametrize("out_layout,f64", [(0, False), (1, False), (1, True)])
def test_prefaulted_new_outputs_equal_device_path(torch_cuda, out_layout, f64):
    """Host calls whose outputs total >= 8 MiB fault the caller's new output arrays in ahead of
    the copies (rsp_hostpool.h Prefaulter, 2 MiB blocks, huge-page advice): 24 CPIs of 64 x 1024
    (9.4 MiB of float / byte outputs, 25 MiB as doubles) through the chunked DMA pipeline, into
    fresh arrays and into reused arrays pre-filled with garbage, both layouts and the double
    outputs -- all bit-exact against the device path, call after call."""
    torch = torch_cuda
    import ctypes as C
    from rsp import _capi as capi
    from rsp import presets, synth
    eng = _engine(64, 1024)
    cf = presets.default_cfar(eng.spec)
    cp = cf.to_c()
    V, Ro = eng.shape
    B = 24
    lib = eng.lib
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)   # noqa: E731
    echo = synth.echo_numpy(eng.spec, B, seed=2024).astype(np.complex64)
    want = _dev(torch, eng, echo, cf)
    if out_layout == capi.RSP_COLMAJOR:
        want = tuple(np.ascontiguousarray(np.swapaxes(w, 1, 2)) for w in want)
    col = np.ascontiguousarray(np.swapaxes(echo.astype(np.complex128), 1, 2))
    oshape = want[0].shape
    dt = (np.float64, np.float64) if f64 else (np.float32, np.uint8)
    reused = (np.full(oshape, 3.0, dt[0]), np.full(oshape, 9, dt[1]), np.full(oshape, 9, dt[1]))
    for call in range(3):
        for outs in ((np.empty(oshape, dt[0]), np.empty(oshape, dt[1]), np.empty(oshape, dt[1])), reused):
            fn = lib.rsp_pc_mtd_cfar_f64 if f64 else lib.rsp_pc_mtd_cfar
            assert fn(eng.ctx, ptr(col), capi.RSP_C128, capi.RSP_COLMAJOR, 64, 1024, B, C.byref(cp), ptr(outs[0]),
                      out_layout, ptr(outs[1]), ptr(outs[2])) == 0
            for g, w in zip(outs, want):
                assert np.array_equal(g, w.astype(g.dtype)), call
    eng.close()

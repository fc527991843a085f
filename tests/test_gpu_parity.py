"""GPU parity of the HIP product path (through the C ABI) against the fp64 oracles.

Bars (written here): RDM rel-err <= 1e-5 (Frobenius) vs the fp64 oracle on
the same synthetic echo; CFAR flags identical except cells whose oracle decision is within
1e-5 relative of its threshold ("near-threshold", counted, bounded).  Integer/index work
(layouts, batching, chunking) must be bit-exact.
"""
import numpy as np
import pytest

import rsp_ref as ref
from _util import MAX_TOL, NEAR_TOL, RDM_TOL, flag_mismatch, max_rel, oracle_flags, oracle_flags_c, oracle_rdm, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _engine(name, P, R, chunk=0):
    from rsp import presets
    from rsp.engine import Engine
    return Engine(presets.make(name, P, R), device=0, chunk=chunk)


def _echo(eng, batch, seed=1001):
    from rsp import synth
    return synth.echo_numpy(eng.spec, batch, seed=seed)


# ---------------------------------------------------------------- pulse compression alone
@pytest.mark.parametrize("name,P,R", [("v2", 64, 1024), ("v2", 128, 4096), ("dmx", 64, 4096), ("legacy", 48, 1031),
                                      ("v2", 16, 16384), ("v2", 16, 12000)])
def test_pc_parity(torch_cuda, name, P, R):
    torch = torch_cuda
    eng = _engine(name, P, R)
    echo = _echo(eng, 2)
    d_in = torch.from_numpy(echo).cuda()
    d_pc = torch.empty((2, P, R), dtype=torch.complex64, device="cuda")
    eng.pc_dev(d_in, d_pc)
    torch.cuda.synchronize()
    got = d_pc.cpu().numpy()
    e64 = echo.astype(np.complex128)
    for b in range(2):
        if name == "v2":
            rp = ref.v2_params(P, R)
            _, p2, p3 = ref.v2_pulses(rp)
            want = ref.fun_lss_pulse_compression(e64[b], p2, p3, 228, 723, R - 951, fir_shift=True)
        elif name == "legacy":
            from rsp import presets
            want = ref.fun_lss_pulse_compression(e64[b], presets.load_data("legacy_pulse2"),
                                                 presets.load_data("legacy_pulse3"), 82, 242, R - 324,
                                                 fir_shift=False, offset2=75, offset3=160)
        else:
            from rsp import presets
            H = ref.dmx_matched_filter(presets.load_data("refDDCDataMF1"), R)
            want = ref.dmx_pulse_compression(e64[b], 0, R, H)
        err = np.linalg.norm(got[b] - want) / np.linalg.norm(want)
        assert err < RDM_TOL, (name, b, err)


@pytest.mark.parametrize("R", [16384, 12000])
def test_pc_overlap_save_matches_whole_transform(torch_cuda, R):
    """The 16384-point segment runs as overlap-save blocks of 4096 (pc_overlap_save); the
    whole-length transform (rsp_set_pc_split(ctx, 0)) must give the same correlation to fp32
    rounding, and every column outside the split segment bit-identically."""
    torch = torch_cuda
    P = 16
    outs = []
    for ols in (1, 0):
        eng = _engine("v2", P, R)
        eng.set_pc_split(ols)
        echo = _echo(eng, 1, seed=77)
        d_in = torch.from_numpy(echo).cuda()
        d_pc = torch.empty((1, P, R), dtype=torch.complex64, device="cuda")
        eng.pc_dev(d_in, d_pc)
        torch.cuda.synchronize()
        outs.append(d_pc.cpu().numpy())
        eng.close()
    a, b = outs
    assert np.array_equal(a[..., :951], b[..., :951])
    err = np.linalg.norm(a - b) / np.linalg.norm(b)
    assert err < 2e-6, err


# ---------------------------------------------------------------- PC -> MTD -> 0-v
@pytest.mark.parametrize("name,P,R,batch", [("v2", 64, 1024, 3), ("v2", 128, 4096, 4), ("dmx", 128, 4096, 2),
                                            ("v2", 256, 8192, 2), ("v2", 512, 16384, 1), ("legacy", 96, 1031, 2),
                                            ("dmx", 32, 512, 3)])
def test_pc_mtd_parity(torch_cuda, name, P, R, batch):
    torch = torch_cuda
    eng = _engine(name, P, R)
    echo = _echo(eng, batch)
    d_in = torch.from_numpy(echo).cuda()
    d_rdm = torch.empty((batch, P, R), dtype=torch.float32, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm)
    torch.cuda.synchronize()
    got = d_rdm.cpu().numpy()
    want = oracle_rdm(name, echo)
    err = rel_err(got, want)
    assert err < RDM_TOL, err
    assert max_rel(got, want) < MAX_TOL, max_rel(got, want)
    # the zero-velocity rows are exactly zero
    lo, hi = ref.zero_v_rows(P, 150)
    assert np.all(got[:, lo:hi, :] == 0)


# ---------------------------------------------------------------- full chain with CFAR
@pytest.mark.parametrize("name,P,R,batch", [("v2", 64, 1024, 2), ("v2", 128, 4096, 3), ("dmx", 128, 4096, 2),
                                            ("legacy", 96, 1031, 1)])
def test_chain_cfar_parity(torch_cuda, name, P, R, batch):
    torch = torch_cuda
    from rsp import presets
    eng = _engine(name, P, R)
    cf = presets.default_cfar(eng.spec)
    echo = _echo(eng, batch)
    d_in = torch.from_numpy(echo).cuda()
    shp = (batch, P, R)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    d_fv = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, flagV=d_fv, cfar=cf)
    torch.cuda.synchronize()
    rdm = oracle_rdm(name, echo)
    assert rel_err(d_rdm.cpu().numpy(), rdm) < RDM_TOL
    flag, flagV, amb = oracle_flags(rdm, cf)
    hard, soft = flag_mismatch(d_flag.cpu().numpy(), flag, amb)
    hardv, softv = flag_mismatch(d_fv.cpu().numpy(), flagV, amb)
    assert hard == 0 and hardv == 0, (hard, hardv)
    assert soft <= max(2, flag.size // 100000) and softv <= max(2, flag.size // 100000), (soft, softv)
    assert flag.sum() > 0 and flagV.sum() > flag.sum()


def test_cfar_standalone_matches_oracle(torch_cuda):
    """rsp_cfar (executeCFAR / fun_CFARflag) on a given RDM: same input for both sides."""
    from rsp import presets
    from rsp.engine import Engine
    rng = np.random.default_rng(3)
    V, R = 128, 868
    rdm = np.abs(rng.standard_normal((2, V, R)) + 1j * rng.standard_normal((2, V, R))).astype(np.float32)
    rdm[:, 40, 100] = 40.0
    rdm[:, 41, 100] = 30.0
    rdm[:, 90, 500:503] = [20.0, 25.0, 22.0]
    cf = presets.Cfar(TR=4.0, TV=4.0, M0=5, zero_v_div=20, segments=[(0, 82), (82, 318), (318, 868)])
    eng = Engine(presets.dmx(16, 64))
    flag, flagV = eng.cfar(rdm, cf)
    want, wantV, amb = oracle_flags(rdm.astype(np.float64), cf)
    assert flag_mismatch(flag, want, amb)[0] == 0
    assert flag_mismatch(flagV, wantV, amb)[0] == 0
    assert want[:, 40, 100].all() and want.sum() > 2


# ---------------------------------------------------------------- boundary behaviour
def test_host_api_matlab_layout_and_dtypes(torch_cuda):
    """rsp_pc_mtd_cfar host path: MATLAB column-major complex double in, column-major out;
    identical to the row-major complex64 device path (conversion is exact)."""
    torch = torch_cuda
    from rsp import _capi as capi, presets
    eng = _engine("v2", 64, 1024)
    cf = presets.default_cfar(eng.spec)
    echo = _echo(eng, 2)
    rdm_r, flag_r, fv_r = eng.pc_mtd_cfar(echo, cf)                       # complex64 row-major
    col = np.ascontiguousarray(np.swapaxes(echo.astype(np.complex128), 1, 2))   # [b][R][P]
    rdm_c, flag_c, fv_c = eng.pc_mtd_cfar(col, cf, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR)
    np.testing.assert_array_equal(np.swapaxes(rdm_c, 1, 2), rdm_r)
    np.testing.assert_array_equal(np.swapaxes(flag_c, 1, 2), flag_r)
    np.testing.assert_array_equal(np.swapaxes(fv_c, 1, 2), fv_r)
    d_in = torch.from_numpy(echo).cuda()
    d_rdm = torch.empty((2, 64, 1024), dtype=torch.float32, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_rdm.cpu().numpy(), rdm_r)


def test_fp16_input_parity(torch_cuda):
    """fp16 I/Q storage, fp32 compute: parity against the oracle fed the same fp16 samples."""
    torch = torch_cuda
    from rsp import synth
    eng = _engine("v2", 128, 4096)
    echo = _echo(eng, 2)
    half = synth.to_half_iq(echo)
    d_in = torch.from_numpy(half).cuda()
    d_rdm = torch.empty((2, 128, 4096), dtype=torch.float32, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm)
    torch.cuda.synchronize()
    e16 = half[..., 0].astype(np.float64) + 1j * half[..., 1].astype(np.float64)
    assert rel_err(d_rdm.cpu().numpy(), oracle_rdm("v2", e16)) < RDM_TOL


def test_batch_and_chunk_invariance(torch_cuda):
    """A CPI's outputs do not depend on its batch neighbours or on the chunk size (bit-exact)."""
    torch = torch_cuda
    from rsp import presets
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    from rsp.engine import Engine
    from rsp import synth
    echo = synth.echo_numpy(spec, 7, seed=77)
    d_in = torch.from_numpy(echo).cuda()
    outs = []
    for chunk in (1, 3, 7):
        eng = Engine(spec, chunk=chunk)
        r = torch.empty((7, 128, 4096), dtype=torch.float32, device="cuda")
        f = torch.empty((7, 128, 4096), dtype=torch.uint8, device="cuda")
        eng.run_dev(d_in, rdm=r, flag=f, cfar=cf)
        torch.cuda.synchronize()
        outs.append((r.cpu().numpy(), f.cpu().numpy()))
        eng.close()
    for r, f in outs[1:]:
        np.testing.assert_array_equal(r, outs[0][0])
        np.testing.assert_array_equal(f, outs[0][1])
    eng = Engine(spec)
    r1 = torch.empty((1, 128, 4096), dtype=torch.float32, device="cuda")
    eng.run_dev(d_in[4:5].contiguous(), rdm=r1)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r1.cpu().numpy()[0], outs[0][0][4])


def test_matlab_mirror(torch_cuda):
    """rsp.matlab keeps the reference's names, argument meaning and outputs."""
    from rsp import matlab, presets, synth
    P, R = 64, 1024
    params = presets.radar_params(P, R)
    spec = presets.v2(P, R)
    echo = synth.echo_numpy(spec, 1, seed=5)[0].astype(np.complex128)
    got = matlab.fun_MTD_produce(echo, params)
    want = ref.fun_MTD_produce_v2(echo, ref.v2_params(P, R))
    assert got.shape == (P, R) and got.dtype == np.float64
    assert rel_err(got, want) < RDM_TOL
    M0 = ref.mtd_zero_num(P, params["wavelength"], params["prf"])
    w32 = want.astype(np.float32).astype(np.float64)
    f, fv = matlab.executeCFAR(w32, 5, 7, 5, 0, 5, 7, 5, 0, M0, 1)
    wf, wfv, amb = ref.executeCFAR(w32, 5, 7, 5, 0, 5, 7, 5, 0, M0, 1, near_tol=NEAR_TOL)
    assert f.dtype == np.float64 and f.shape == (P, R)
    assert flag_mismatch(f, wf, amb)[0] == 0 and flag_mismatch(fv, wfv, amb)[0] == 0
    cf = matlab.fun_CFARflag(w32, 5, 7, 5, 0, 5, 7, 5, 0, M0, 1, segments=((0, 228), (228, 951), (951, 1024)))
    wcf, _, amb2 = ref.fun_CFARflag(w32, 5, 7, 5, 0, 5, 7, 5, 0, M0, 1,
                                    segments=((1, 228), (229, 951), (952, 1024)), near_tol=NEAR_TOL)
    assert flag_mismatch(cf, wcf, amb2)[0] == 0


def test_error_behaviour(torch_cuda):
    from rsp import RspError, _capi as capi, presets
    from rsp.engine import Engine
    eng = _engine("v2", 64, 1024)
    with pytest.raises(ValueError):          # echo of the wrong shape (host-side check)
        eng.pc_mtd(np.zeros((1, 64, 1000), np.complex64))
    a = np.zeros((1, 64, 1000), np.complex64)  # and the C ABI's own check
    out = np.empty((1, 64, 1000), np.float32)
    rc = eng.lib.rsp_pc_mtd(eng.ctx, a.ctypes.data, capi.RSP_C64, capi.RSP_ROWMAJOR, 64, 1000, 1,
                            out.ctypes.data, capi.RSP_ROWMAJOR)
    assert rc == capi.RSP_ERR_SHAPE and b"context was created" in eng.lib.rsp_last_error(eng.ctx)
    # MATLAB raises an index error when the Doppler window does not fit: so does the ABI
    cf = presets.Cfar(M0=20)                 # 64 - 41 = 23 Doppler cells < 24
    with pytest.raises(RspError) as ei:
        eng.pc_mtd_cfar(_echo(eng, 1), cf)
    assert ei.value.code == capi.RSP_ERR_CFAR_WINDOW
    with pytest.raises(RspError) as ei:      # no radix plan and beyond the Bluestein range
        Engine(presets.v2(1100, 1024))
    assert ei.value.code == capi.RSP_ERR_UNSUPPORTED


def test_full_batch_properties(torch_cuda):
    """c3 size (128 x 4096, batch 1024): spot CPIs against the C oracle, and the exact
    size-independent property RDM(2x) = 2 RDM(x) (power-of-two scaling is exact in fp32)."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec)
    B = 1024
    echo = synth.echo_torch(spec, B, seed=2024)
    rdm = torch.empty((B, 128, 4096), dtype=torch.float32, device="cuda")
    flag = torch.empty((B, 128, 4096), dtype=torch.uint8, device="cuda")
    eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    idx = [0, 511, 1023]
    sample = echo[idx].cpu().numpy()
    want = oracle_rdm("v2", sample)
    assert rel_err(rdm[idx].cpu().numpy(), want) < RDM_TOL
    wflag, _, amb = oracle_flags(want, cf)
    assert flag_mismatch(flag[idx].cpu().numpy(), wflag, amb)[0] == 0
    rdm2 = torch.empty_like(rdm)
    flag2 = torch.empty_like(flag)
    echo.mul_(2.0)
    eng.run_dev(echo, rdm=rdm2, flag=flag2, cfar=cf)
    torch.cuda.synchronize()
    assert torch.equal(rdm2, rdm * 2.0)
    assert torch.equal(flag2, flag)


def test_create_legacy_matches_python_preset(torch_cuda):
    """rsp_create_legacy (the one-argument MEX path: split and FIR in C, the measured pulses
    passed in) builds the same context as the Python legacy preset: bit-identical RDMs."""
    import ctypes as C
    from rsp import _capi as capi, presets, synth
    from rsp.engine import Engine
    P, R = 48, 1031
    lib = capi.load_library()
    ctx = C.c_void_p()
    p2 = presets.load_data("legacy_pulse2").astype(np.complex128)
    p3 = presets.load_data("legacy_pulse3").astype(np.complex128)
    arrs = [np.ascontiguousarray(a) for a in (p2.real, p2.imag, p3.real, p3.imag)]
    dp = [a.ctypes.data_as(C.POINTER(C.c_double)) for a in arrs]
    assert lib.rsp_create_legacy(C.byref(ctx), 0, P, R, dp[0], dp[1], len(p2), dp[2], dp[3], len(p3)) == 0
    echo = synth.echo_numpy(presets.legacy(P, R), 2, seed=19).astype(np.complex128)
    out = np.empty((2, P, R), np.float32)
    rc = lib.rsp_pc_mtd(ctx, echo.ctypes.data, capi.RSP_C128, capi.RSP_ROWMAJOR, P, R, 2, out.ctypes.data,
                        capi.RSP_ROWMAJOR)
    assert rc == 0
    lib.rsp_destroy(ctx)
    with Engine(presets.legacy(P, R)) as eng:
        want = eng.pc_mtd(echo)
    np.testing.assert_array_equal(out, want)
    assert lib.rsp_create_legacy(C.byref(ctx), 0, P, 300, dp[0], dp[1], len(p2), dp[2], dp[3], len(p3)) != 0


def test_create_v2_matches_python_preset(torch_cuda):
    """rsp_create_v2 (the MEX path: params fields -> context in C) == the Python v2 preset."""
    import ctypes as C
    from rsp import _capi as capi, presets, synth
    from rsp.engine import Engine
    P, R = 64, 1024
    lib = capi.load_library()
    ctx = C.c_void_p()
    pp = (C.c_int64 * 4)(R, 228, 723, R - 951)
    tao = (C.c_double * 3)(0.16e-6, 8e-6, 28e-6)
    assert lib.rsp_create_v2(C.byref(ctx), 0, P, R, pp, 25e6, 20e6, tao) == 0
    echo = synth.echo_numpy(presets.v2(P, R), 2, seed=9).astype(np.complex128)
    out = np.empty((2, P, R), np.float32)
    rc = lib.rsp_pc_mtd(ctx, echo.ctypes.data, capi.RSP_C128, capi.RSP_ROWMAJOR, P, R, 2, out.ctypes.data,
                        capi.RSP_ROWMAJOR)
    assert rc == 0
    lib.rsp_destroy(ctx)
    with Engine(presets.v2(P, R)) as eng:
        want = eng.pc_mtd(echo)
    assert rel_err(out, want) < 1e-6
    assert rel_err(out, oracle_rdm("v2", echo)) < RDM_TOL


@pytest.mark.parametrize("P,R", [(256, 3000), (512, 2048)])
def test_chain_cfar_tile_mappings(torch_cuda, P, R):
    """MTD tiles narrower than a cache line (W = 16) are grouped 4 per XCD when the tile count
    is a multiple of 32 (512 x 2048: 128 tiles) and mapped in order otherwise (256 x 3000: 188
    tiles, R % 16 != 0 so the flag background is written per cell): both against the oracle."""
    torch = torch_cuda
    from rsp import presets
    eng = _engine("v2", P, R)
    cf = presets.default_cfar(eng.spec)
    echo = _echo(eng, 2)
    d_in = torch.from_numpy(echo).cuda()
    shp = (2, P, R)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, cfar=cf)
    torch.cuda.synchronize()
    rdm = oracle_rdm("v2", echo)
    assert rel_err(d_rdm.cpu().numpy(), rdm) < RDM_TOL
    flag, _, amb = oracle_flags_c(rdm, cf)
    hard, soft = flag_mismatch(d_flag.cpu().numpy(), flag, amb)
    assert hard == 0, (hard, soft)
    assert soft <= max(2, flag.size // 100000), soft
    assert flag.sum() > 0


def test_range_groups_across_group_boundaries(torch_cuda):
    """The grouped range stage (rsp_capi.cpp run_chain_body: the range CFAR of up to 16 chunks of a
    pipeline in one launch, hit indices relative to the group's first output cell): 37 one-CPI
    chunks on two pipelines (groups of 16 + a partial group each), 8 chunks of 5 with a short last
    chunk, and one 37-CPI chunk give the same RDM and flags, bit for bit."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(64, 1024)
    cf = presets.default_cfar(spec)
    B = 37
    echo = synth.echo_numpy(spec, B, seed=3737)
    d_in = torch.from_numpy(echo).cuda()
    V, Ro = spec.V, spec.R_out
    outs = []
    for chunk in (1, 5, 37):
        eng = Engine(spec, chunk=chunk)
        r = torch.empty((B, V, Ro), dtype=torch.float32, device="cuda")
        f = torch.empty((B, V, Ro), dtype=torch.uint8, device="cuda")
        eng.run_dev(d_in, rdm=r, flag=f, cfar=cf)
        torch.cuda.synchronize()
        outs.append((r.cpu().numpy(), f.cpu().numpy()))
        eng.close()
    assert outs[0][1].sum() > 0
    for r, f in outs[1:]:
        np.testing.assert_array_equal(r, outs[0][0])
        np.testing.assert_array_equal(f, outs[0][1])


# ---------------------------------------------------------------- fun_lss_range_concate (main.m)
def test_legacy_range_concat_chain(torch_cuda):
    """main.m's legacy simulation chain (MatlabProcess_xuzerui/main.m:206-211): PC, then
    fun_lss_range_concate (fun_lss_range_concate.m:4-7: 1031 -> 868 columns), then MTD + 0-v and
    fun_CFARflag's 1:82 | 83:318 | 319:868 split (main_cfar.m:143-145), which assumes the 868
    columns.  rsp_set_range_concat gathers the PC columns between PC and MTD: the RDM against the
    numpy oracle of the concatenated chain, CFAR flags against the oracle's, and -- the gather
    being a copy -- bit-exact against PC without concat, gathered, then MTD / CFAR of those rows."""
    torch = torch_cuda
    from rsp import presets
    from rsp.engine import Engine
    P, R, B = 96, 1031, 2
    spec = presets.legacy(P, R, concat=True)
    assert spec.R_out == 868 and spec.cfar_segments[-1] == (318, 868)
    cf = presets.default_cfar(spec)
    eng = Engine(spec)
    echo = _echo(eng, B, seed=1211)
    d_in = torch.from_numpy(echo).cuda()
    shp = (B, P, 868)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, cfar=cf)
    torch.cuda.synchronize()
    p2, p3 = presets.load_data("legacy_pulse2"), presets.load_data("legacy_pulse3")
    want = np.stack([ref.fun_MTD_produce_legacy(x.astype(np.complex128), p2, p3, concat=True) for x in echo])
    got = d_rdm.cpu().numpy()
    assert rel_err(got, want) < RDM_TOL
    flag, _, amb = oracle_flags(want, cf)
    hard, soft = flag_mismatch(d_flag.cpu().numpy(), flag, amb)
    assert hard == 0 and soft <= 2, (hard, soft)
    assert flag.sum() > 0
    # PC alone returns the concatenated rows = the plain legacy PC rows gathered (bit-exact)
    plain = Engine(presets.legacy(P, R))
    pc_full = torch.empty((B, P, R), dtype=torch.complex64, device="cuda")
    plain.pc_dev(d_in, pc_full)
    pc_cat = torch.empty((B, P, 868), dtype=torch.complex64, device="cuda")
    eng.pc_dev(d_in, pc_cat)
    torch.cuda.synchronize()
    gathered = torch.cat([pc_full[..., a:a + n] for a, n in presets.LEGACY_CONCAT], dim=-1).contiguous()
    assert torch.equal(pc_cat, gathered)
    # the MTD / CFAR stage on those rows (rsp_mtd_cfar_dev) gives the chain's outputs exactly
    r2 = torch.empty(shp, dtype=torch.float32, device="cuda")
    f2 = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.mtd_dev(gathered, rdm=r2, flag=f2, cfar=cf)
    torch.cuda.synchronize()
    assert torch.equal(r2, d_rdm) and torch.equal(f2, d_flag)
    # host API (MATLAB layout) through the same context: identical
    rdm_h, flag_h, _ = eng.pc_mtd_cfar(echo, cf)
    assert np.array_equal(rdm_h, got) and np.array_equal(flag_h, d_flag.cpu().numpy())
    # a part outside the PC row is refused; no parts restores the PC width (the plain legacy chain)
    from rsp import _capi as capi
    import ctypes as C
    bad = (C.c_int64 * 1)(1000), (C.c_int64 * 1)(100)
    assert eng.lib.rsp_set_range_concat(eng.ctx, 1, bad[0], bad[1]) == capi.RSP_ERR_ARG
    eng.set_range_concat([])
    eng.spec = presets.legacy(P, R)
    r3 = torch.empty((B, P, R), dtype=torch.float32, device="cuda")
    eng.run_dev(d_in, rdm=r3)
    r4 = torch.empty((B, P, R), dtype=torch.float32, device="cuda")
    plain.run_dev(d_in, rdm=r4)
    torch.cuda.synchronize()
    assert torch.equal(r3, r4)
    eng.close()
    plain.close()

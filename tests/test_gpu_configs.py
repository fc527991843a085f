"""GPU parity at the BASELINE configs the other files do not cover, through the C ABI, against
the fp64 oracles (SURVEY.md §8d bars, written below):

  c4   256 x 8192 sliding-window stream (MTD/main_produce_dataset_win_xzr_v2.m:94-144):
       2 frame pairs x 4 windows, executeCFAR with M0 = 11
  c5   512 x 16384 fp16 I/Q with fp32 compute + CFAR (M0 = 22), plus the fp16 tolerance
       sweep over input scale and SNR against the oracle fed the UNQUANTISED echo
  v2 native 13-beam window stream: 332 x 3404 x 13 beams x 4 windows (rows 0/83/166/249,
       :37-38,109-139), Bluestein MTD + window slicing
  legacy native 1536 x 1031 (MatlabProcess_xuzerui/fun_MTD_produce.m:3-126,
       main_produce_dataset_win_xzr.m:31-40), whose slow-time window is read back and pinned
       to the reference's kaiser_win.mat
  the fused chain with SO and non-default reference / guard windows (executeCFAR.m:1-93 with
       the runtime-window MTD kernel and the generic range stage)

Bars: RDM ||d||_F / ||ref||_F <= 1e-5 against fp64 on the same (fp32-representable) samples;
CFAR flags identical outside the near-threshold band (|x - T avg| / (T avg) < 1e-5, counted).
fp16 storage (c5) against the unquantised echo: RDM rel-err <= FP16_RDM_TOL and flags identical
outside a near-threshold band of FP16_NEAR_TOL, over the stated usable input range.
"""
import json
import os

import numpy as np
import pytest

from _util import NEAR_TOL, RDM_TOL, flag_mismatch, oracle_flags_c, oracle_rdm, rel_err

pytestmark = pytest.mark.gpu

# fp16 I/Q storage: 10 explicit mantissa bits, rounding error <= 2^-11 relative per component.
# The storage error of the RDM (fp64 oracle on the fp16 samples vs on the unquantised echo) is
# white quantisation noise of the +30 dB clutter spread over every Doppler bin: measured
# 1.7e-4 (SNR 30 dB) .. 9.7e-4 (SNR 0 dB) over the usable range, hence the 2e-3 bar.
FP16_RDM_TOL = 2e-3
FP16_NEAR_TOL = 1e-3
FP16_MIN_NORMAL = 2.0 ** -14
FP16_MAX = 65504.0

@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _mround(x):
    return int(np.floor(x + 0.5))


def _windows(frames, win):
    """[beams, F+1, P, R] -> [beams, F, win, P, R] by the reference's slicing (v2.m:120-133)."""
    beams, nf1, P, R = frames.shape
    out = np.empty((beams, nf1 - 1, win, P, R), dtype=frames.dtype)
    for b in range(beams):
        for n in range(nf1 - 1):
            pair = np.concatenate([frames[b, n], frames[b, n + 1]], axis=0)
            for i in range(win):
                s = _mround(i * P / win)
                out[b, n, i] = pair[s:s + P]
    return out


def _window_check(torch, spec, frames, win, cf):
    """Window stream vs (a) the plain chain on the sliced echo (bit-exact) and (b) the fp64
    oracle on the sliced echo (bars above)."""
    from rsp.engine import Engine
    beams, nf1, P, R = frames.shape
    nf = nf1 - 1
    eng = Engine(spec, device=0)
    d_frames = torch.from_numpy(frames).cuda()
    shp = (beams, nf, win, spec.V, spec.R_out)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.window_dev(d_frames, win, rdm=d_rdm, flag=d_flag, cfar=cf)
    sliced = _windows(frames, win).reshape(-1, P, R)
    n = sliced.shape[0]
    d_sl = torch.from_numpy(np.ascontiguousarray(sliced)).cuda()
    e_rdm = torch.empty((n, spec.V, spec.R_out), dtype=torch.float32, device="cuda")
    e_flag = torch.empty((n, spec.V, spec.R_out), dtype=torch.uint8, device="cuda")
    eng.run_dev(d_sl, rdm=e_rdm, flag=e_flag, cfar=cf)
    torch.cuda.synchronize()
    assert torch.equal(d_rdm.reshape(n, spec.V, -1), e_rdm)
    assert torch.equal(d_flag.reshape(n, spec.V, -1), e_flag)
    got = d_rdm.cpu().numpy().reshape(n, spec.V, -1)
    gflag = d_flag.cpu().numpy().reshape(n, spec.V, -1)
    eng.close()
    del d_sl, e_rdm, e_flag, d_frames
    rdm = oracle_rdm(spec.name, sliced)
    err = rel_err(got, rdm)
    assert err < RDM_TOL, err
    flag, _, amb = oracle_flags_c(rdm, cf)
    hard, soft = flag_mismatch(gflag, flag, amb)
    assert hard == 0, (hard, soft)
    assert soft <= max(2, flag.size // 100000), soft
    assert flag.sum() > 0
    return err, int(flag.sum()), soft


def test_c4_window_stream_parity(torch_cuda):
    """c4: 256 x 8192, 2 frame pairs x 4 windows (starts 0/64/128/192), CFAR with M0 = 11."""
    from rsp import presets, synth
    P, R, win = 256, 8192, 4
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    assert cf.M0 == 11
    frames = synth.echo_numpy(spec, 3, seed=1044).reshape(1, 3, P, R)
    _window_check(torch_cuda, spec, frames, win, cf)


def test_v2_native_13_beam_window_stream(torch_cuda):
    """v2 native: 332 x 3404 per beam, 13 beams, one frame pair, 4 windows starting at rows
    0/83/166/249 -- the MTD_win_all_beams loop of main_produce_dataset_win_xzr_v2.m:109-139
    (Bluestein slow-time DFT for P = 332)."""
    from rsp import presets, synth
    P, R, win, beams = 332, 3404, 4, 13
    assert [_mround(i * P / win) for i in range(win)] == [0, 83, 166, 249]
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    frames = synth.echo_numpy(spec, beams * 2, seed=1313).reshape(beams, 2, P, R)
    _window_check(torch_cuda, spec, frames, win, cf)


def test_legacy_native_chain_and_kaiser_pin(torch_cuda):
    """Legacy native 1536 x 1031 (MatlabProcess_xuzerui/fun_MTD_produce.m:3-126): the chain with
    fun_CFARflag's hard-coded segments against the fp64 oracle, and the product's own
    kaiser(1536, 8) read back through the MTD kernel and pinned to kaiser_win.mat: a slow-time
    impulse at pulse p0 in range column r gives |X[k]| = w[p0] for every Doppler bin k."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    P, R = 1536, 1031
    spec = presets.legacy(P, R)
    eng = Engine(spec, device=0)
    cf = presets.default_cfar(spec)
    echo = synth.echo_numpy(spec, 1, seed=1536)
    d_in = torch.from_numpy(echo).cuda()
    d_rdm = torch.empty((1, P, R), dtype=torch.float32, device="cuda")
    d_flag = torch.empty((1, P, R), dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, cfar=cf)
    # window read-back: CPI b, column r carries the impulse at pulse r + b*R
    pc = np.zeros((2, P, R), np.complex64)
    for b in range(2):
        for r in range(R):
            p0 = r + b * R
            if p0 < P:
                pc[b, p0, r] = 1.0
    d_pc = torch.from_numpy(pc).cuda()
    d_w = torch.empty((2, P, R), dtype=torch.float32, device="cuda")
    eng.mtd_dev(d_pc, rdm=d_w)
    torch.cuda.synchronize()
    rdm = oracle_rdm("legacy", echo)
    assert rel_err(d_rdm.cpu().numpy(), rdm) < RDM_TOL
    flag, _, amb = oracle_flags_c(rdm, cf)
    hard, soft = flag_mismatch(d_flag.cpu().numpy(), flag, amb)
    assert hard == 0 and soft <= 2, (hard, soft)
    golden = np.load(os.path.join(os.path.dirname(__file__), "golden", "kaiser_win_1536_beta8.npy"))
    wv = d_w.cpu().numpy()
    live = np.ones(P, bool)
    import rsp_ref as ref
    lo, hi = ref.zero_v_rows(P, 150)
    live[lo:hi] = False                                  # fun_0v_pressing rows are zeroed
    got = np.empty(P)
    for p0 in range(P):
        b, r = divmod(p0, R)
        col = wv[b, live, r]
        assert np.ptp(col) <= 1e-6 * col.max()   # flat over Doppler
        got[p0] = col.mean()
    np.testing.assert_allclose(got, golden, rtol=1e-6, atol=0)
    eng.close()


@pytest.mark.parametrize("methodV,methodR,ref_n,guard,P,R", [(1, 1, 5, 7, 128, 4096), (0, 0, 3, 2, 128, 4096),
                                                            (1, 0, 8, 4, 64, 1024), (0, 1, 5, 7, 64, 1024),
                                                            (1, 1, 3, 2, 256, 8192), (0, 0, 5, 4, 128, 4096)])
def test_chain_cfar_variants(torch_cuda, methodV, methodR, ref_n, guard, P, R):
    """The fused hot path (Doppler CFAR in the MTD kernel, range stage on its hit list) with
    SO (method 1) and reference / guard windows other than the default 5 / 7 -- the runtime-
    window MTD kernel (also for 5 reference cells with a guard other than 7: the compiled-in
    window is 5 + 7 only) and the generic hit-region range stage -- against the oracle."""
    torch = torch_cuda
    import dataclasses
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(P, R)
    cf = dataclasses.replace(presets.default_cfar(spec), methodV=methodV, methodR=methodR, refV=ref_n, saveV=guard,
                             refR=ref_n, saveR=guard, TV=4.0, TR=4.0)
    eng = Engine(spec, device=0)
    echo = synth.echo_numpy(spec, 2, seed=2000 + ref_n + guard)
    d_in = torch.from_numpy(echo).cuda()
    shp = (2, P, R)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    d_fv = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, flagV=d_fv, cfar=cf)
    torch.cuda.synchronize()
    rdm = oracle_rdm("v2", echo)
    assert rel_err(d_rdm.cpu().numpy(), rdm) < RDM_TOL
    flag, flagV, amb = oracle_flags_c(rdm, cf)
    hard, soft = flag_mismatch(d_flag.cpu().numpy(), flag, amb)
    hardv, softv = flag_mismatch(d_fv.cpu().numpy(), flagV, amb)
    assert hard == 0 and hardv == 0, (hard, hardv)
    assert soft <= 4 and softv <= 4, (soft, softv)
    assert flag.sum() > 0 and flagV.sum() >= flag.sum()
    eng.close()


@pytest.mark.parametrize("P,R,W", [(128, 4096, 32), (256, 2048, 16), (512, 2048, 16)])
def test_dense_hit_regions_range_stage(torch_cuda, P, R, W):
    """The range stage of executeCFAR.m:45-84 on dense hit regions: thresholds of 1.5 make most
    tiles carry more than 64 Doppler hits, so the wave-per-region range kernel (regions of
    <= 4096 cells: its first-64 batch and its per-hit tail loop) and the workgroup-per-region
    one (P = 512) both run past their first pass; flags against the oracle as above."""
    torch = torch_cuda
    import dataclasses
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(P, R)
    cf = dataclasses.replace(presets.default_cfar(spec), TV=1.5, TR=1.5)
    eng = Engine(spec, device=0)
    echo = synth.echo_numpy(spec, 2, seed=3000 + P)
    d_in = torch.from_numpy(echo).cuda()
    shp = (2, P, R)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    d_fv = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, flagV=d_fv, cfar=cf)
    torch.cuda.synchronize()
    rdm = oracle_rdm("v2", echo)
    assert rel_err(d_rdm.cpu().numpy(), rdm) < RDM_TOL
    flag, flagV, amb = oracle_flags_c(rdm, cf)
    # hits per MTD tile (W range bins x all Doppler rows): the dense case this test is about
    per_tile = flagV.reshape(2, P, R // W, W).sum(axis=(1, 3))
    assert (per_tile > 64).mean() > 0.5, per_tile.max()
    hard, soft = flag_mismatch(d_flag.cpu().numpy(), flag, amb)
    hardv, softv = flag_mismatch(d_fv.cpu().numpy(), flagV, amb)
    assert hard == 0 and hardv == 0, (hard, hardv)
    assert soft <= 8 and softv <= 8, (soft, softv)
    assert flag.sum() > 0
    eng.close()


# ---------------------------------------------------------------- c5: fp16 I/Q at 512 x 16384
def _fp16_run(torch, eng, echo, cf):
    from rsp import synth
    half = synth.to_half_iq(echo)
    d_in = torch.from_numpy(half).cuda()
    shp = (echo.shape[0], eng.spec.V, eng.spec.R_out)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, cfar=cf)
    torch.cuda.synchronize()
    return half, d_rdm.cpu().numpy(), d_flag.cpu().numpy()


def test_c5_fp16_chain_parity(torch_cuda):
    """c5: one CPI of fp16 I/Q at 512 x 16384 through PC -> MTD -> CFAR (M0 = 22).  Against the
    oracle fed the same fp16 samples (compute error: the fp32 bars); against the unquantised
    echo (storage + compute error: the fp16 bars)."""
    from rsp import presets, synth
    from rsp.engine import Engine
    P, R = 512, 16384
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    assert cf.M0 == 22
    eng = Engine(spec, device=0)
    echo = synth.echo_numpy(spec, 1, seed=1005, dtype=np.complex128)
    half, got, gflag = _fp16_run(torch_cuda, eng, echo, cf)
    eng.close()
    e16 = half[..., 0].astype(np.float64) + 1j * half[..., 1].astype(np.float64)
    rdm16 = oracle_rdm("v2", e16)
    assert rel_err(got, rdm16) < RDM_TOL
    flag16, _, amb16 = oracle_flags_c(rdm16, cf)
    hard, soft = flag_mismatch(gflag, flag16, amb16)
    assert hard == 0 and soft <= max(2, flag16.size // 100000), (hard, soft)
    rdm = oracle_rdm("v2", echo)
    assert rel_err(got, rdm) < FP16_RDM_TOL
    flag, _, amb = oracle_flags_c(rdm, cf, near_tol=FP16_NEAR_TOL)
    hard, soft = flag_mismatch(gflag, flag, amb)
    assert hard <= max(2, int(flag.sum()) // 100000), (hard, soft)
    assert flag.sum() > 0


def fp16_sweep(torch, P=512, R=16384, scales=(2.0 ** -18, 2.0 ** -14, 2.0 ** -10, 1.0, 2.0 ** 8, 2.0 ** 10, 2.0 ** 12),
               snrs=(0.0, 10.0, 20.0, 30.0)):
    """fp16 tolerance sweep (north_star config 5) over input scale and target SNR.  Per row:
      compute error  GPU vs the fp64 oracle fed the SAME fp16 samples (the kernel's parity);
      storage error  the fp64 oracle on the fp16 samples vs on the unquantised echo (what fp16
                     I/Q costs by itself);
      end to end     GPU vs the fp64 oracle on the unquantised echo (near band FP16_NEAR_TOL).
    `usable`: every |I|, |Q| x scale below the fp16 maximum and the noise sigma x scale above
    the smallest normal."""
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    rows = []
    for snr in snrs:
        echo = synth.echo_numpy(spec, 1, seed=1500 + int(snr), dtype=np.complex128, snr_db=snr)
        peak = float(max(np.abs(echo.real).max(), np.abs(echo.imag).max()))
        rdm = oracle_rdm("v2", echo)
        flag, _, amb = oracle_flags_c(rdm, cf, near_tol=FP16_NEAR_TOL)
        for sc in scales:
            half, got, gflag = _fp16_run(torch, eng, echo * sc, cf)
            usable = peak * sc < FP16_MAX and np.sqrt(0.5) * sc >= FP16_MIN_NORMAL
            row = dict(snr_db=snr, scale=sc, usable=bool(usable), flags_ref=int(flag.sum()))
            fin = np.isfinite(got)
            row["nonfinite"] = int((~fin).sum())
            if fin.all():
                e16 = half[..., 0].astype(np.float64) + 1j * half[..., 1].astype(np.float64)
                rdm16 = oracle_rdm("v2", e16)
                f16, _, amb16 = oracle_flags_c(rdm16, cf)
                row["compute_rel_err"] = rel_err(got, rdm16)
                row["compute_flag_hard"], row["compute_flag_soft"] = flag_mismatch(gflag, f16, amb16)
                row["storage_rel_err"] = rel_err(rdm16, rdm * sc)
                row["storage_flag_flips"] = int((f16 != flag).sum())
                row["rdm_rel_err"] = rel_err(got, rdm * sc)
                row["flag_hard"], row["flag_soft"] = flag_mismatch(gflag, flag, amb)
            rows.append(row)
    eng.close()
    return rows


def test_fp16_tolerance_sweep(torch_cuda):
    """The sweep at c5 size.  Bars: the compute error meets the fp32 bars at every finite row;
    in the usable range the end-to-end RDM error stays below FP16_RDM_TOL and flags flip only
    inside the FP16_NEAR_TOL band (at most max(2, 1e-5 of the flags) outside it); the ends
    behave as fp16 predicts.  The table goes to gpurun_out/fp16_sweep.json."""
    rows = fp16_sweep(torch_cuda)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "fp16_sweep.json"), "w") as f:
        json.dump(dict(P=512, R=16384, rdm_tol=FP16_RDM_TOL, near_tol=FP16_NEAR_TOL, rows=rows), f, indent=1)
    for r in rows:
        print(r)
    for r in rows:
        if r["nonfinite"] == 0:
            assert r["compute_rel_err"] < RDM_TOL and r["compute_flag_hard"] == 0, r
        if r["usable"]:
            assert r["nonfinite"] == 0, r
            assert r["rdm_rel_err"] < FP16_RDM_TOL and r["storage_rel_err"] < FP16_RDM_TOL, r
            assert r["flag_hard"] <= max(2, r["flags_ref"] // 100000), r
    assert sum(r["usable"] for r in rows) >= 12
    # subnormal noise loses precision (the storage error grows > 2x over the same SNR's usable
    # rows); overflowing samples make the RDM non-finite
    for r in rows:
        if r["scale"] == 2.0 ** -18:
            base = min(q["storage_rel_err"] for q in rows if q["snr_db"] == r["snr_db"] and q["usable"])
            assert r["storage_rel_err"] > 2.0 * base, r
    assert all(r["nonfinite"] > 0 for r in rows if r["scale"] == 2.0 ** 12)


# ---------------------------------------------------------------- full BASELINE sizes
def test_c5_full_batch_properties(torch_cuda):
    """c5 at the bench's full size (64 fp16 CPIs of 512 x 16384: 64 one-CPI chunks through both
    pipelines, overlap-save PC): spot CPIs against the oracle fed the same fp16 samples, and the
    exact size-independent property RDM(2x) = 2 RDM(x), flags unchanged (scaling fp16 I/Q by 2
    is exact, and so is every fp32 operation after it)."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    P, R, B = 512, 16384, 64
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    echo = synth.echo_torch(spec, B, seed=2025, half=True)
    rdm = torch.empty((B, P, R), dtype=torch.float32, device="cuda")
    flag = torch.empty((B, P, R), dtype=torch.uint8, device="cuda")
    eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    for i in (0, 37, 63):
        h = echo[i].cpu().numpy().astype(np.float64)
        want = oracle_rdm("v2", (h[..., 0] + 1j * h[..., 1])[None])
        assert rel_err(rdm[i].cpu().numpy()[None], want) < RDM_TOL, i
        wflag, _, amb = oracle_flags_c(want, cf)
        hard, soft = flag_mismatch(flag[i].cpu().numpy()[None], wflag, amb)
        assert hard == 0 and soft <= max(2, wflag.size // 100000), (i, hard, soft)
    rdm2 = torch.empty_like(rdm)
    flag2 = torch.empty_like(flag)
    echo.mul_(2.0)
    eng.run_dev(echo, rdm=rdm2, flag=flag2, cfar=cf)
    torch.cuda.synchronize()
    assert torch.equal(rdm2, rdm * 2.0)
    assert torch.equal(flag2, flag)
    eng.close()


def test_c4_full_stream_properties(torch_cuda):
    """c4 at the bench's full size (32 frame pairs x 4 windows of 256 x 8192): spot windows
    against the oracle on the sliced echo, and RDM(2x) = 2 RDM(x) with flags unchanged."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    P, R, F, W = 256, 8192, 32, 4
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    frames = synth.echo_torch(spec, F + 1, seed=2026).reshape(1, F + 1, P, R)
    shp = (1, F, W, P, R)
    rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.window_dev(frames, W, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    for n, i in ((0, 0), (17, 3), (31, 2)):
        s = _mround(i * P / W)
        pair = torch.cat([frames[0, n], frames[0, n + 1]], dim=0)[s:s + P].cpu().numpy()
        want = oracle_rdm("v2", pair[None])
        assert rel_err(rdm[0, n, i].cpu().numpy()[None], want) < RDM_TOL, (n, i)
        wflag, _, amb = oracle_flags_c(want, cf)
        hard, soft = flag_mismatch(flag[0, n, i].cpu().numpy()[None], wflag, amb)
        assert hard == 0 and soft <= max(2, wflag.size // 100000), (n, i, hard, soft)
    rdm2 = torch.empty_like(rdm)
    flag2 = torch.empty_like(flag)
    frames.mul_(2.0)
    eng.window_dev(frames, W, rdm=rdm2, flag=flag2, cfar=cf)
    torch.cuda.synchronize()
    assert torch.equal(rdm2, rdm * 2.0)
    assert torch.equal(flag2, flag)
    eng.close()

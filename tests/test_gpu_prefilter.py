"""GPU parity of the echo pre-filters (rsp_prefilter_dev) against the fp64
restatement (oracle/prefilter_ref.py).  Bar: max |gpu - ref| / max |ref| <= 1e-6 (fp32
products of fp32 inputs; the MTI difference is one fp32 subtraction, the gain one multiply),
the zero rows exact; iSTC may run in place, MTI may not."""
import numpy as np
import pytest

import prefilter_ref as pr

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def pf():
    import torch
    assert torch.cuda.is_available()
    from rsp.prefilter import Prefilter
    p = Prefilter(0)
    yield p
    p.close()


def _echo(rng, *shape):
    return (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)


def _close(got, want):
    return np.abs(got - want).max() <= TOL * np.abs(want).max()


@pytest.mark.parametrize("P,R", [(128, 4096), (64, 1024), (40, 1030), (30, 64)])
def test_mti_parity(pf, P, R):
    import torch
    x = _echo(np.random.default_rng(P + R), 3, P, R)
    y = pf.apply_dev(x, mti_lag=30)
    torch.cuda.synchronize()
    y = y.cpu().numpy()
    for b in range(3):
        want = pr.fun_Process_MTI(x[b].astype(np.complex128))
        assert (y[b, max(P - 30, 0):] == 0).all()
        if P > 30:
            assert _close(y[b], want)


def test_istc_and_both(pf):
    import torch
    P, R = 128, 4096
    rng = np.random.default_rng(7)
    x = _echo(rng, 2, P, R)
    ini = rng.uniform(-30, 10, 1025)                       # a 1025-point curve as the reference's
    stc, y = pf.fun_iSTC(x[0], ini)
    torch.cuda.synchronize()
    _, want = pr.fun_iSTC(x[0].astype(np.complex128), ini)
    assert _close(y.cpu().numpy(), want)
    from rsp.prefilter import istc_gain
    _, g = istc_gain(ini, R)
    both = pf.apply_dev(x, gain=g, mti_lag=30)
    torch.cuda.synchronize()
    for b in range(2):
        _, w = pr.fun_iSTC(pr.fun_Process_MTI(x[b].astype(np.complex128)), ini)
        assert _close(both[b].cpu().numpy(), w)
    # in place (gain only)
    d = torch.from_numpy(x).cuda()
    pf.apply_dev(d, out=d, gain=g)
    torch.cuda.synchronize()
    assert _close(d[1].cpu().numpy(), pr.fun_iSTC(x[1].astype(np.complex128), ini)[1])


def test_mti_in_place_refused_and_odd_R(pf):
    import torch
    from rsp import RspError
    d = torch.zeros((64, 64), dtype=torch.complex64, device="cuda")
    with pytest.raises(RspError):
        pf.apply_dev(d, out=d, mti_lag=30)
    with pytest.raises(RspError):
        pf.apply_dev(torch.zeros((64, 63), dtype=torch.complex64, device="cuda"), mti_lag=30)


def test_prefilter_then_chain(pf):
    """MTI ahead of the v2 chain (the pre-filter feeding Engine.run_dev on the device): the
    chain's RDM of the filtered echo matches the C oracle's RDM of the oracle-filtered echo
    (rel-err <= 1e-5, the chain's bar)."""
    import torch
    from _util import oracle_rdm, rel_err
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    eng = Engine(spec, device=0)
    echo = synth.echo_numpy(spec, 1, seed=1003)
    f = pf.apply_dev(torch.from_numpy(echo).cuda(), mti_lag=30)
    rdm = torch.empty((1, 128, 4096), dtype=torch.float32, device="cuda")
    eng.run_dev(f, rdm=rdm)
    torch.cuda.synchronize()
    fe = pr.fun_Process_MTI(echo[0].astype(np.complex128))[None]
    assert rel_err(rdm.cpu().numpy(), oracle_rdm("v2", fe)) < 1e-5
    eng.close()


def _fused_case(torch, name, P, R, batch, gain_on, lag, half=False, seed=1101):
    """RDM / flags of the chain with the pre-filters fused (rsp_set_prefilter), and the fp64
    oracle's for the oracle-filtered echo (MTI, then iSTC: they commute)."""
    from _util import oracle_flags, oracle_rdm
    from rsp import presets, synth
    from rsp.engine import Engine
    from rsp.prefilter import istc_gain
    eng = Engine(presets.make(name, P, R), device=0)
    cf = presets.default_cfar(eng.spec)
    echo = synth.echo_numpy(eng.spec, batch, seed=seed)
    g = None
    if gain_on:
        ini = np.random.default_rng(seed).uniform(-30, 10, min(1025, R))
        _, g = istc_gain(ini, R)
    eng.set_prefilter(gain=g, mti_lag=lag)
    if half:
        src = synth.to_half_iq(echo)
        d_in = torch.from_numpy(src).cuda()
        e64 = src[..., 0].astype(np.float64) + 1j * src[..., 1].astype(np.float64)
    else:
        d_in = torch.from_numpy(echo).cuda()
        e64 = echo.astype(np.complex128)
    shp = (batch, eng.spec.V, eng.spec.R_out)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, cfar=cf)
    torch.cuda.synchronize()
    fe = np.stack([pr.fun_Process_MTI(e64[b], lag) if lag else e64[b] for b in range(batch)])
    if g is not None:
        fe = fe * np.asarray(g, np.float64)[None, None, :]
    rdm = oracle_rdm(name, fe)
    flag, _, amb = oracle_flags(rdm, cf)
    eng.close()
    return d_rdm.cpu().numpy(), d_flag.cpu().numpy(), rdm, flag, amb


@pytest.mark.parametrize("name,P,R,batch,gain_on,lag", [("v2", 128, 4096, 2, True, 30), ("v2", 128, 4096, 1, False, 30),
                                                        ("v2", 64, 1024, 2, True, 0), ("dmx", 64, 4096, 1, True, 7),
                                                        ("v2", 64, 16384, 1, True, 5)])
def test_fused_prefilter_chain_parity(name, P, R, batch, gain_on, lag):
    """Pre-filters fused into the chain (iSTC in PC's echo load, MTI in the MTD's load of the
    PC rows) against the fp64 oracle of the explicitly filtered echo: the chain's bars (RDM
    rel-err <= 1e-5, no flag mismatch outside the near-threshold band)."""
    import torch
    from _util import RDM_TOL, flag_mismatch, rel_err
    got, gflag, rdm, flag, amb = _fused_case(torch, name, P, R, batch, gain_on, lag)
    assert rel_err(got, rdm) < RDM_TOL
    hard, soft = flag_mismatch(gflag, flag, amb)
    assert hard == 0 and soft <= max(2, flag.size // 100000), (hard, soft)


def test_fused_prefilter_fp16_input():
    """fp16 I/Q echo with the fused gain and MTI: the oracle is fed the same fp16 samples."""
    import torch
    from _util import RDM_TOL, rel_err
    got, _, rdm, _, _ = _fused_case(torch, "v2", 128, 4096, 1, True, 30, half=True)
    assert rel_err(got, rdm) < RDM_TOL


def test_fused_prefilter_bluestein_mti():
    """MTI fused into the Bluestein MTD (the v2 native P = 332)."""
    import torch
    from _util import RDM_TOL, rel_err
    got, _, rdm, _, _ = _fused_case(torch, "v2", 332, 3404, 1, True, 30)
    assert rel_err(got, rdm) < RDM_TOL


def test_fused_prefilter_off_is_identity():
    """set_prefilter(None, 0) restores the unfiltered chain bit for bit."""
    import torch
    from rsp import presets, synth
    from rsp.engine import Engine
    eng = Engine(presets.v2(64, 1024), device=0)
    echo = torch.from_numpy(synth.echo_numpy(eng.spec, 1, seed=3)).cuda()
    outs = []
    for g, lag in ((None, 0), (np.full(1024, 0.5, np.float32), 30), (None, 0)):
        eng.set_prefilter(gain=g, mti_lag=lag)
        r = torch.empty((1, 64, 1024), dtype=torch.float32, device="cuda")
        eng.run_dev(echo, rdm=r)
        torch.cuda.synchronize()
        outs.append(r.cpu().numpy())
    assert np.array_equal(outs[0], outs[2]) and not np.array_equal(outs[0], outs[1])
    eng.close()

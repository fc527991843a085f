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

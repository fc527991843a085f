"""The fused one-launch chain (chain_kernel, rsp_set_fused) against the chunked two-kernel
pipeline and the fp64 oracle.

The fused path computes the same arithmetic as pc_persist_kernel + mtd_kernel +
cfar_hits_kernel (same FFT code, same operation order), so every output must be bit-identical
to the chunked pipeline's; rsp_chain_check must report no expired in-kernel wait.
"""
import numpy as np
import pytest

from _util import RDM_TOL, flag_mismatch, oracle_flags, oracle_rdm, rel_err

pytestmark = pytest.mark.gpu

P, R = 128, 4096


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _run(torch, eng, d_in, batch, cfar, want_rdm=True, want_fv=False):
    shp = (batch, P, R)
    rdm = torch.empty(shp, dtype=torch.float32, device="cuda") if want_rdm else None
    flag = torch.empty(shp, dtype=torch.uint8, device="cuda") if cfar is not None else None
    fv = torch.empty(shp, dtype=torch.uint8, device="cuda") if want_fv else None
    eng.run_dev(d_in, rdm=rdm, flag=flag, flagV=fv, cfar=cfar)
    torch.cuda.synchronize()
    eng.chain_check()
    cpu = lambda t: t.cpu().numpy() if t is not None else None   # noqa: E731
    return cpu(rdm), cpu(flag), cpu(fv)


def _pair(torch, batch, cfar=True, want_rdm=True, want_fv=False, half=False, seed=5):
    """(fused outputs, chunked outputs, echo) for one input."""
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec) if cfar else None
    echo = synth.echo_numpy(spec, batch, seed=seed)
    src = synth.to_half_iq(echo) if half else echo
    d_in = torch.from_numpy(src).cuda()
    outs = []
    for fused in (1, 0):
        with Engine(spec) as eng:
            eng.set_fused(fused)
            outs.append(_run(torch, eng, d_in, batch, cf, want_rdm, want_fv))
    return outs[0], outs[1], echo, cf


def _same(a, b):
    for x, y in zip(a, b):
        if x is None or y is None:
            assert x is None and y is None
        else:
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("batch", [1, 5, 8, 19, 64])
def test_fused_matches_chunked(torch_cuda, batch):
    """Bit-identical RDM and flags for batches that leave some of the 8 queues empty or
    uneven (1, 5, 19) and for whole ring turns (64 = 8 queues x 8 CPIs)."""
    f, c, _, _ = _pair(torch_cuda, batch)
    _same(f, c)
    assert f[1].sum() > 0


def test_fused_oracle_parity(torch_cuda):
    """Fused chain against the fp64 oracle: RDM rel-err <= 1e-5, flags equal away from ties."""
    (rdm, flag, _), _, echo, cf = _pair(torch_cuda, 3, seed=11)
    want = oracle_rdm("v2", echo)
    assert rel_err(rdm, want) < RDM_TOL
    wf, _, amb = oracle_flags(want, cf)
    hard, soft = flag_mismatch(flag, wf, amb)
    assert hard == 0 and soft <= 2, (hard, soft)
    assert wf.sum() > 0


def test_fused_variants(torch_cuda):
    """No CFAR; flagV requested; flags without an RDM output (internal RDM ring); fp16 I/Q."""
    torch = torch_cuda
    f, c, _, _ = _pair(torch, 11, cfar=False)
    _same(f, c)
    f, c, _, _ = _pair(torch, 11, want_fv=True)
    _same(f, c)
    assert f[2].sum() > f[1].sum()
    f, c, _, _ = _pair(torch, 27, want_rdm=False)
    _same(f, c)
    f, c, _, _ = _pair(torch, 9, half=True)
    _same(f, c)


def test_fused_full_batch(torch_cuda):
    """c3 size (1024 CPIs): fused and chunked agree bit for bit on the whole batch."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    B = 1024
    d_in = synth.echo_torch(spec, B, seed=1234, device=torch.device("cuda"))
    res = []
    for fused in (1, 0):
        with Engine(spec) as eng:
            eng.set_fused(fused)
            rdm = torch.empty((B, P, R), dtype=torch.float32, device="cuda")
            flag = torch.empty((B, P, R), dtype=torch.uint8, device="cuda")
            eng.run_dev(d_in, rdm=rdm, flag=flag, cfar=cf)
            torch.cuda.synchronize()
            eng.chain_check()
            res.append((rdm, flag))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])

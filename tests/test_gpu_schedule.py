"""The chunk schedule of the chain at the v2 128 x 4096 shape (c2/c3): chunks of CPIs on one,
two (the default) or three stream pipelines, each with its own PC scratch slot, the range stage
of a chunk run inside the next MTD launch of its pipeline.  The schedule only changes which
launches overlap, so the outputs must be BIT-identical across pipeline counts and chunkings (a
remainder chunk, two chunks, many), with and without CFAR and flagV, fp32 and fp16 input, the
fused pre-filters, and the internal RDM (flags-only calls); and within the chain's bars
against the fp64 oracle (MTD/fun_MTD_produce.m:12-158, CFAR_WangCai/executeCFAR.m:1-93)."""
import numpy as np
import pytest

from _util import NEAR_TOL, RDM_TOL, flag_mismatch, oracle_flags_c, oracle_rdm, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _chain(torch, spec, echo, cfar, streams, chunk, flagv=True, prefilter=False):
    from rsp.engine import Engine
    eng = Engine(spec, device=0, chunk=chunk, streams=streams)
    if prefilter:
        eng.set_prefilter(gain=np.linspace(0.5, 2.0, spec.R).astype(np.float32), mti_lag=30)
    B = echo.shape[0]
    shp = (B, spec.V, spec.R_out)
    rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    flag = torch.empty(shp, dtype=torch.uint8, device="cuda") if cfar else None
    fv = torch.empty(shp, dtype=torch.uint8, device="cuda") if (cfar and flagv) else None
    eng.run_dev(echo, rdm=rdm, flag=flag, flagV=fv, cfar=cfar)
    torch.cuda.synchronize()
    out = (rdm.cpu().numpy(), None if flag is None else flag.cpu().numpy(), None if fv is None else fv.cpu().numpy())
    eng.close()
    return out


@pytest.mark.parametrize("batch,chunk,cfar_on,flagv,half,prefilter", [
    (10, 4, True, True, False, False),     # 3 chunks, a remainder chunk of 2
    (8, 4, True, False, False, False),     # two chunks, one per pipeline
    (40, 0, True, False, False, False),    # the default 16-CPI chunks: 3 chunks
    (12, 3, False, False, False, False),   # PC -> MTD only (c2)
    (9, 4, True, True, True, False),       # fp16 I/Q input
    (10, 4, True, False, False, True),     # fused iSTC + MTI
])
def test_schedule_bit_exact(torch_cuda, batch, chunk, cfar_on, flagv, half, prefilter):
    torch = torch_cuda
    from rsp import presets, synth
    spec = presets.v2(128, 4096)
    cfar = presets.default_cfar(spec) if cfar_on else None
    echo = synth.echo_torch(spec, batch, seed=1700 + batch, device="cuda", half=half)
    dflt = _chain(torch, spec, echo, cfar, 0, chunk, flagv, prefilter)      # default (two pipelines)
    three = _chain(torch, spec, echo, cfar, 3, chunk, flagv, prefilter)     # three pipelines
    one = _chain(torch, spec, echo, cfar, 1, chunk, flagv, prefilter)       # one stream
    for a, b, c in zip(dflt, three, one):
        if a is None:
            assert b is None and c is None
            continue
        assert np.array_equal(a, b)
        assert np.array_equal(a, c)
    if cfar_on:
        assert dflt[1].sum() > 0


def test_schedule_vs_oracle(torch_cuda):
    """The default schedule against the fp64 oracle (RDM <= 1e-5, flags outside the near-
    threshold band identical) on CPIs spread over three chunks."""
    torch = torch_cuda
    from rsp import presets, synth
    spec = presets.v2(128, 4096)
    cfar = presets.default_cfar(spec)
    echo = synth.echo_numpy(spec, 6, seed=1777)
    d = torch.from_numpy(echo).cuda()
    rdm, flag, _ = _chain(torch, spec, d, cfar, 0, 2, flagv=False)
    for b in (0, 3, 5):
        ref = oracle_rdm("v2", echo[b:b + 1])[0]
        assert rel_err(rdm[b], ref) < RDM_TOL
        want, _, amb = oracle_flags_c(ref[None], cfar, near_tol=NEAR_TOL)
        bad, near = flag_mismatch(flag[b], want[0], amb[0])
        assert bad == 0, (b, bad, near)


def test_internal_rdm(torch_cuda):
    """No RDM output requested (flags only): the internal RDM slots give the flags of the
    full-output call."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cfar = presets.default_cfar(spec)
    echo = synth.echo_torch(spec, 7, seed=1790, device="cuda")
    eng = Engine(spec, device=0, chunk=2)
    shp = (7, spec.V, spec.R_out)
    rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    f1 = torch.empty(shp, dtype=torch.uint8, device="cuda")
    f2 = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(echo, rdm=rdm, flag=f1, cfar=cfar)
    eng.run_dev(echo, rdm=None, flag=f2, cfar=cfar)
    torch.cuda.synchronize()
    eng.close()
    assert torch.equal(f1, f2) and int(f1.sum()) > 0

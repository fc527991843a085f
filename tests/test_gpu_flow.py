"""The persistent dataflow schedule (rsp_set_flow 1 / 2: PC rows, MTD tiles and range-CFAR jobs
as work items of per-XCD queues in ONE launch, hand-offs through counters in memory) against the
chunked two-pipeline schedule (mode 0): the same kernels' arithmetic on the same inputs, so the
RDM, flag and flagV planes must be bit-identical -- at batch sizes that leave queues empty (1, 5),
uneven (19) or deep (64: eight CPIs per queue, every ring slot reused), with and without CFAR,
fp16 I/Q input, and an RDM-less call (the RDM ring).  No hand-off wait may hit its bound."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _run(torch, eng, echo, cf, flow, want_rdm=True, want_fv=True):
    eng.set_flow(flow)
    B = echo.shape[0]
    V, Ro = eng.shape
    rdm = torch.full((B, V, Ro), float("nan"), dtype=torch.float32, device="cuda") if want_rdm else None
    flag = torch.full((B, V, Ro), 7, dtype=torch.uint8, device="cuda") if cf is not None else None
    fv = torch.full((B, V, Ro), 7, dtype=torch.uint8, device="cuda") if (cf is not None and want_fv) else None
    eng.run_dev(echo, rdm=rdm, flag=flag, flagV=fv, cfar=cf)
    torch.cuda.synchronize()
    if flow:
        assert eng.flow_status() == 0, "a dataflow hand-off wait hit its bound"
    return [t.cpu().numpy() if t is not None else None for t in (rdm, flag, fv)]


@pytest.mark.parametrize("B", [1, 5, 19, 64])
@pytest.mark.parametrize("flow", [1, 2])
def test_flow_matches_chunked(torch_cuda, B, flow):
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    echo = synth.echo_torch(spec, B, seed=500 + B, device=torch_cuda.device("cuda", 0))
    want = _run(torch_cuda, eng, echo, cf, 0)
    got = _run(torch_cuda, eng, echo, cf, flow)
    for g, w, name in zip(got, want, ("rdm", "flag", "flagV")):
        assert np.array_equal(g, w, equal_nan=False), name
    assert want[1].sum() > 0
    # PC + MTD only (config c2)
    want = _run(torch_cuda, eng, echo, None, 0)
    got = _run(torch_cuda, eng, echo, None, flow)
    assert np.array_equal(got[0], want[0])
    eng.close()


def test_flow_fp16_and_rdm_ring(torch_cuda):
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    echo = synth.echo_torch(spec, 24, seed=4242, device=torch.device("cuda", 0), half=True)
    want = _run(torch, eng, echo, cf, 0)
    got = _run(torch, eng, echo, cf, 1)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    # no RDM output: the range stage reads the dataflow's RDM ring
    got = _run(torch, eng, echo, cf, 2, want_rdm=False, want_fv=False)
    assert np.array_equal(got[1], want[1])
    eng.close()


def test_flow_repeated_calls(torch_cuda):
    """Back-to-back dataflow calls reuse the rings and the control block (zeroed per launch)."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    outs = []
    for seed in (1, 2, 1):
        echo = synth.echo_torch(spec, 16, seed=seed, device=torch.device("cuda", 0))
        outs.append(_run(torch, eng, echo, cf, 2))
    for g, w in zip(outs[0], outs[2]):
        assert np.array_equal(g, w)
    assert not np.array_equal(outs[0][0], outs[1][0])
    eng.close()

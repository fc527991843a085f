"""Multi-context / multi-stream behaviour of the C ABI (rsp.h threading model):

  - two host threads, each owning a context on device 0 and its own stream, run the c3 chain
    concurrently; outputs are bit-identical to a single-thread run (the per-device launch
    setup is thread-safe, nothing is shared between contexts);
  - one context used from two streams back to back: the second call's stream waits for the
    first call's use of the context scratch, so both results are bit-identical to
    sequential calls;
  - rsp_cfar at R = 16384 with rFlag = 0 (the copy path needs no LDS), and a range window the
    LDS-staged kernel cannot hold is refused with RSP_ERR_UNSUPPORTED instead of a launch
    failure.
"""
import threading

import numpy as np
import pytest

from _util import flag_mismatch, oracle_flags_c

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _run(torch, eng, d_in, cf, stream=None):
    B, P, R = d_in.shape
    rdm = torch.empty((B, P, R), dtype=torch.float32, device="cuda")
    flag = torch.empty((B, P, R), dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=rdm, flag=flag, cfar=cf, stream=stream)
    return rdm, flag


def test_two_threads_two_contexts(torch_cuda):
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    inputs = [synth.echo_torch(spec, 96, seed=s) for s in (31, 32)]
    torch.cuda.synchronize()
    want = []
    with Engine(spec, device=0) as eng:
        for d in inputs:
            r, f = _run(torch, eng, d, cf)
            torch.cuda.synchronize()
            want.append((r, f))
    got = [None, None]
    errs = []

    def worker(i):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with Engine(spec, device=0) as eng:
                outs = []
                for _ in range(3):           # repeated calls interleave with the other thread
                    with torch.cuda.stream(s):
                        outs.append(_run(torch, eng, inputs[i], cf, stream=s))
                s.synchronize()
                got[i] = outs
        except Exception as e:               # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for i in range(2):
        for r, f in got[i]:
            assert torch.equal(r, want[i][0]) and torch.equal(f, want[i][1])


def test_one_context_two_streams(torch_cuda):
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    a = synth.echo_torch(spec, 64, seed=41)
    b = synth.echo_torch(spec, 64, seed=42)
    torch.cuda.synchronize()
    with Engine(spec, device=0) as eng:
        ra, fa = _run(torch, eng, a, cf)
        torch.cuda.synchronize()
        rb, fb = _run(torch, eng, b, cf)
        torch.cuda.synchronize()
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for _ in range(3):
            with torch.cuda.stream(s1):
                r1, f1 = _run(torch, eng, a, cf, stream=s1)
            with torch.cuda.stream(s2):
                r2, f2 = _run(torch, eng, b, cf, stream=s2)
            s1.synchronize()
            s2.synchronize()
            assert torch.equal(r1, ra) and torch.equal(f1, fa)
            assert torch.equal(r2, rb) and torch.equal(f2, fb)


def test_cfar_wide_rows(torch_cuda):
    from rsp import presets
    from rsp._capi import RSP_ERR_UNSUPPORTED, RspError
    from rsp.engine import Engine
    rng = np.random.default_rng(16)
    V, R = 64, 16384
    rdm = np.abs(rng.standard_normal((1, V, R)) + 1j * rng.standard_normal((1, V, R))).astype(np.float32)
    rdm[0, 30, 5000] = 60.0
    rdm[0, 31, 9000:9002] = [40.0, 45.0]
    eng = Engine(None)
    for rflag, ref_n, guard in ((0, 3, 2), (1, 5, 7), (0, 5, 7)):
        cf = presets.Cfar(refR=ref_n, saveR=guard, refV=ref_n, saveV=guard, TR=4.0, TV=4.0, M0=2, rFlag=rflag,
                          zero_v_div=0)
        flag, flagV = eng.cfar(rdm, cf)
        want, wantV, amb = oracle_flags_c(rdm.astype(np.float64), cf)
        assert flag_mismatch(flag, want, amb)[0] == 0 and flag_mismatch(flagV, wantV, amb)[0] == 0
        assert want[0, 30, 5000] == 1
    cf = presets.Cfar(refR=3, saveR=2, refV=3, saveV=2, M0=2, rFlag=1, zero_v_div=0)
    with pytest.raises(RspError) as ei:      # the LDS-staged range kernel cannot hold 16384 cells
        eng.cfar(rdm, cf)
    assert ei.value.code == RSP_ERR_UNSUPPORTED
    ok = presets.Cfar(refR=3, saveR=2, refV=3, saveV=2, TR=4.0, TV=4.0, M0=2, rFlag=1, zero_v_div=0)
    flag, _ = eng.cfar(rdm[:, :, :16000].copy(), ok)    # 16000 cells still fit
    want, _, amb = oracle_flags_c(rdm[:, :, :16000].astype(np.float64), ok)
    assert flag_mismatch(flag, want, amb)[0] == 0
    eng.close()

"""Golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py from the numpy
oracle): both oracles must keep reproducing them (CPU), and the GPU path must match them
within the §8d bars (gpu)."""
import os

import numpy as np
import pytest

import coracle
import rsp_ref as ref
from _util import RDM_TOL, flag_mismatch, rel_err

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = [("v2_32x1024", "v2"), ("dmx_32x512", "dmx"), ("legacy_48x1031", "legacy")]


def _load(case):
    return np.load(os.path.join(G, case + ".npz"))


@pytest.mark.parametrize("case,name", CASES)
def test_c_oracle_reproduces_golden(case, name):
    d = _load(case)
    echo = d["echo"]
    P, R = echo.shape
    rdm = coracle.pc_mtd(echo[None].astype(np.complex128), coracle.preset(name, P, R))[0]
    assert rel_err(rdm, d["rdm"]) < 1e-12
    c = dict(refR=5, saveR=7, TR=float(d["T"]), methodR=0, refV=5, saveV=7, TV=float(d["T"]), methodV=0,
             M0=int(d["M0"]), rFlag=1, zero_v_div=20)
    segs0 = [(int(a) - 1, int(b)) for a, b in d["segs"]]
    f, fv = coracle.cfar(d["rdm"], c, segs0)
    np.testing.assert_array_equal(f[0], d["flag"])
    np.testing.assert_array_equal(fv[0], d["flagV"])


def test_numpy_oracle_reproduces_cfar_edges():
    d = np.load(os.path.join(G, "cfar_edges.npz"))
    segs = [tuple(int(x) for x in s) for s in d["segs"]]
    for method in (0, 1):
        f, fv = ref.fun_CFARflag(d["rdm"], 5, 7, 3.0, method, 5, 7, 3.0, method, 2, 1, segments=segs)
        np.testing.assert_array_equal(f, d["flag_m%d" % method])
        np.testing.assert_array_equal(fv, d["flagV_m%d" % method])
    # first maximum wins among equal neighbours (executeCFAR.m:68-70)
    assert d["flag_m0"][20, 70] == 1 and d["flag_m0"][20, 71] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("case,name", CASES)
def test_gpu_matches_golden(case, name):
    from rsp import presets
    from rsp.engine import Engine
    d = _load(case)
    echo = d["echo"]
    P, R = echo.shape
    spec = presets.make(name, P, R)
    cf = presets.Cfar(TR=float(d["T"]), TV=float(d["T"]), M0=int(d["M0"]), zero_v_div=20,
                      segments=[(int(a) - 1, int(b)) for a, b in d["segs"]])
    with Engine(spec) as eng:
        rdm, flag, flagV = eng.pc_mtd_cfar(echo[None], cf)
    assert rel_err(rdm[0], d["rdm"]) < RDM_TOL
    assert flag_mismatch(flag[0], d["flag"], d["amb"])[0] == 0
    assert flag_mismatch(flagV[0], d["flagV"], d["amb"])[0] == 0


@pytest.mark.gpu
def test_gpu_cfar_edges_exact():
    """Same fp32 input on both sides: every decision away from the threshold and every
    first-maximum tie must match."""
    from rsp import presets
    from rsp.engine import Engine
    d = np.load(os.path.join(G, "cfar_edges.npz"))
    segs = [(int(a) - 1, int(b)) for a, b in d["segs"]]
    rdm32 = d["rdm"].astype(np.float32)
    with Engine(presets.dmx(16, 64)) as eng:
        for method in (0, 1):
            cf = presets.Cfar(TR=3.0, TV=3.0, methodR=method, methodV=method, M0=2, zero_v_div=0, segments=segs)
            flag, flagV = eng.cfar(rdm32[None], cf)
            near = d["amb_m%d" % method]
            assert flag_mismatch(flag[0], d["flag_m%d" % method], near)[0] == 0
            assert flag_mismatch(flagV[0], d["flagV_m%d" % method], near)[0] == 0
            if method == 0:
                assert flag[0, 20, 70] == 1 and flag[0, 20, 71] == 0
        cf = presets.Cfar(TR=3.0, TV=3.0, M0=2, rFlag=0, zero_v_div=0, segments=[])
        flag, _ = eng.cfar(rdm32[None], cf)
        assert flag_mismatch(flag[0], d["flag_noR"], d["amb_m0"])[0] == 0

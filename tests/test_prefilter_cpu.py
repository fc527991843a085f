"""Echo pre-filters, CPU side: the loop-faithful fp64 restatement
(oracle/prefilter_ref.py) against closed forms, and the host logic of rsp/prefilter.py (stc
curve reading and zero-padding, the dimension error).  Parity with MATLAB is unpinned: the
reference ships no stc curve and calls neither function."""
import numpy as np
import pytest

import prefilter_ref as pr


def test_mti_closed_form():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((40, 12)) + 1j * rng.standard_normal((40, 12))
    y = pr.fun_Process_MTI(x)
    np.testing.assert_array_equal(y[:10], x[30:] - x[:10])
    assert (y[10:] == 0).all()
    assert (pr.fun_Process_MTI(x[:30]) == 0).all()          # P <= 30: the loop never runs
    np.testing.assert_array_equal(pr.fun_Process_MTI(x, lag=1)[:39], np.diff(x, axis=0))


def test_istc_closed_form_and_padding(tmp_path):
    from rsp.prefilter import istc_gain, read_stc_curve
    rng = np.random.default_rng(2)
    x = rng.standard_normal((4, 16)) + 1j * rng.standard_normal((4, 16))
    ini = np.linspace(-20, 20, 10)
    stc, y = pr.fun_iSTC(x, ini)
    assert stc.shape == (16,) and (stc[10:] == 0).all()
    np.testing.assert_allclose(y, x * 10 ** (stc / 20), rtol=1e-15)
    f = tmp_path / "stc.txt"
    f.write_text("\n".join("%.6f" % v for v in ini) + "\n")
    np.testing.assert_allclose(read_stc_curve(str(f)), ini, atol=1e-6)
    s2, g = istc_gain(str(f), 16)
    np.testing.assert_allclose(s2, stc, atol=1e-6)
    assert g.dtype == np.float32 and g[12] == 1.0
    with pytest.raises(ValueError):
        istc_gain(np.zeros(17), 16)
    with pytest.raises(ValueError):
        pr.fun_iSTC(x, np.zeros(17))

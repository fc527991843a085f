"""A plain C program over the C ABI (tests/native/capi_consumer.c, built by
__graft_entry__.build()): the host-buffer entry points a C / MEX caller binds, in both
layouts and both output types, executeCFAR on the double RDM, a moving point target found on
its Doppler row and flagged, and the error contract -- with no Python in the data path."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "build", "capi_consumer")


def test_c_program_over_the_c_abi():
    assert os.path.exists(EXE), "build() first (make -C tests/native)"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout + r.stderr[-2000:]
    _, row, col, det = r.stdout.split()
    assert int(row) == 20 + 64 and abs(int(col) - 1800) <= 1 and int(det) >= 1

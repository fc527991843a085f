#!/usr/bin/env python3
"""Extract the reference's *data* (not code) into small .npy files.

Run in the build container only (it reads /root/reference, which does not exist on
the GPU box).  Outputs are committed, so nothing at run time touches the reference.

What is extracted and why:
  * MatlabProcess_xuzerui/refDDCDataMF1.mat `refData` (67x1 complex, integer valued):
    the measured long-pulse replica the DMX matched filter loads
    (CFAR_WangCai/DMX_SignalProcessing_main_xzr.m:158). Input of the `dmx` preset.
  * MatlabProcess_xuzerui/refDBFDataMF1.mat `refData`: the alternative replica
    (same file :157, commented out there). Kept for completeness of the preset.
  * The measured pulse2/pulse3 sample tables hard-coded in
    MatlabProcess_xuzerui/fun_MTD_produce.m:54-60 (75 and 160 complex samples):
    inputs of the `legacy` preset. Only the numbers are kept.
  * MatlabProcess_xuzerui/kaiser_win.mat `kaiser_win` = kaiser(1536, 8): the one
    known-answer vector of the reference (golden for the window).

All .mat files are MAT v5 and are read with scipy.io.loadmat (no pickle).
"""
import os
import re
import sys

import numpy as np
import scipy.io

REF = "/root/reference/MatlabProcess_xuzerui"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG_DATA = os.path.join(REPO, "radar-signal-process_amd", "rsp", "data")
GOLDEN = os.path.join(REPO, "tests", "golden")


def _table(text, name):
    m = re.search(name + r"\s*=\s*\[([^\]]*)\]", text)
    if m is None:
        raise RuntimeError("table %s not found" % name)
    return np.array([float(t) for t in m.group(1).replace(",", " ").split()], dtype=np.float64)


def main():
    if not os.path.isdir(REF):
        print("reference not mounted; nothing to do", file=sys.stderr)
        return 1
    os.makedirs(PKG_DATA, exist_ok=True)
    os.makedirs(GOLDEN, exist_ok=True)

    ddc = scipy.io.loadmat(os.path.join(REF, "refDDCDataMF1.mat"))["refData"][:, 0]
    np.save(os.path.join(PKG_DATA, "refDDCDataMF1.npy"), ddc.astype(np.complex128))
    dbf = scipy.io.loadmat(os.path.join(REF, "refDBFDataMF1.mat"))["refData"][:, 0]
    np.save(os.path.join(PKG_DATA, "refDBFDataMF1.npy"), dbf.astype(np.complex128))

    with open(os.path.join(REF, "fun_MTD_produce.m"), "rb") as f:
        text = f.read().decode("latin-1")
    p2 = _table(text, "pulse2_real") + 1j * _table(text, "pulse2_imag")
    p3 = _table(text, "pulse3_real") + 1j * _table(text, "pulse3_imag")
    assert p2.size == 75 and p3.size == 160, (p2.size, p3.size)
    np.save(os.path.join(PKG_DATA, "legacy_pulse2.npy"), p2)
    np.save(os.path.join(PKG_DATA, "legacy_pulse3.npy"), p3)

    kw = scipy.io.loadmat(os.path.join(REF, "kaiser_win.mat"))["kaiser_win"][:, 0]
    np.save(os.path.join(GOLDEN, "kaiser_win_1536_beta8.npy"), kw.astype(np.float64))
    print("ok:", ddc.shape, dbf.shape, p2.shape, p3.shape, kw.shape)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Generate the committed golden vectors (tests/golden/*.npz) from the loop-faithful fp64
numpy oracle (oracle/rsp_ref.py).  Inputs are the deterministic synthetic echoes of
SURVEY.md §8d (numpy PCG64, seed 1000 + config id); outputs are the oracle's fp64 RDM and
CFAR flags.  The reference itself (MATLAB) cannot run here, so these pin the oracle's
behaviour over time and give the GPU path a fixed target; see oracle/rsp_ref.py for how
the oracle itself is pinned (kaiser_win.mat + known-answer tests).

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "radar-signal-process_amd")]

import rsp_ref as ref  # noqa: E402
from rsp import presets, synth  # noqa: E402  (the synthetic-echo recipe only)

OUT = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(ROOT, "radar-signal-process_amd", "rsp", "data")

CASES = [
    # name, preset, P, R, seed
    ("v2_32x1024", "v2", 32, 1024, 1001),
    ("dmx_32x512", "dmx", 32, 512, 1002),
    ("legacy_48x1031", "legacy", 48, 1031, 1003),
]


def chain(name, P, R, echo):
    if name == "v2":
        rp = ref.v2_params(P, R)
        rdm = ref.fun_MTD_produce_v2(echo, rp)
        segs = [(1, 228), (229, 951), (952, R)]
    elif name == "dmx":
        rp = ref.v2_params(P, R)
        rdm = ref.fun_MTD_produce_dmx_syn(echo, np.load(os.path.join(DATA, "refDDCDataMF1.npy")))
        segs = [(1, R)]
    else:
        rp = dict(wavelength=ref.C_LIGHT / 5500e6, prf=1 / 64.88e-6)
        rdm = ref.fun_MTD_produce_legacy(echo, np.load(os.path.join(DATA, "legacy_pulse2.npy")),
                                         np.load(os.path.join(DATA, "legacy_pulse3.npy")))
        segs = [(1, 82), (83, 318), (319, 868)]
    M0 = ref.mtd_zero_num(P, rp["wavelength"], rp["prf"])
    cf = dict(refR=5, saveR=7, TR=4.0, methodR=0, refV=5, saveV=7, TV=4.0, methodV=0, M0=M0, rFlag=1)
    flag, flagV, amb = ref.main_cfar_chain(rdm, cf, segs, 20, near_tol=1e-5)
    return rdm, flag, flagV, amb, cf, segs


def cfar_edge_cases():
    """executeCFAR / fun_CFARflag corner cases: edge fallbacks, spikes next to segment
    boundaries, equal neighbours (first max), constant fields, SO method."""
    rng = np.random.default_rng(99)
    V, R = 64, 120
    base = np.abs(rng.standard_normal((V, R)) + 1j * rng.standard_normal((V, R)))
    m = base.astype(np.float32).astype(np.float64)   # exactly representable in fp32
    m[3, 5] = 60.0          # first used Doppler row, near the left range edge
    m[60, 118] = 60.0       # last used Doppler row region, right edge
    m[30, 39] = 50.0        # segment boundary at 40 (1-based 40|41)
    m[30, 40] = 50.0        # equal neighbours across the boundary
    m[20, 70] = 45.0        # equal neighbours inside a segment: first max wins
    m[20, 71] = 45.0
    m[40:44, 90] = 0.0      # zeros
    segs = [(1, 40), (41, 120)]
    out = {}
    for method in (0, 1):
        f, fv, amb = ref.fun_CFARflag(m, 5, 7, 3.0, method, 5, 7, 3.0, method, 2, 1, segments=segs, near_tol=1e-5)
        out["flag_m%d" % method], out["flagV_m%d" % method], out["amb_m%d" % method] = f, fv, amb
    f0, fv0 = ref.executeCFAR(m, 5, 7, 3.0, 0, 5, 7, 3.0, 0, 2, 0)
    out["flag_noR"] = f0
    return m, segs, out


def main():
    for case, name, P, R, seed in CASES:
        spec = presets.make(name, P, R)
        echo = synth.echo_numpy(spec, 1, seed=seed)[0]          # complex64 input
        rdm, flag, flagV, amb, cf, segs = chain(name, P, R, echo.astype(np.complex128))
        np.savez_compressed(os.path.join(OUT, case + ".npz"), echo=echo, rdm=rdm, flag=flag.astype(np.uint8),
                            flagV=flagV.astype(np.uint8), amb=amb, M0=cf["M0"], T=cf["TR"],
                            segs=np.array(segs, np.int64))
        print(case, "rdm max %.3g flags %d flagV %d ambiguous %d" % (rdm.max(), flag.sum(), flagV.sum(), amb.sum()))
    m, segs, out = cfar_edge_cases()
    np.savez_compressed(os.path.join(OUT, "cfar_edges.npz"), rdm=m, segs=np.array(segs, np.int64),
                        **{k: (v.astype(np.uint8) if v.dtype != bool else v) for k, v in out.items()})
    print("cfar_edges", {k: int(v.sum()) for k, v in out.items()})


if __name__ == "__main__":
    main()

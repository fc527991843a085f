"""Shared helpers for the parity tests: oracle-side references for a preset and the
comparison rules of SURVEY.md §8d."""
import numpy as np

import coracle
import rsp_ref as ref

RDM_TOL = 1e-5        # ||RDM_gpu - RDM_ref||_F / ||RDM_ref||_F   (north_star)
NEAR_TOL = 1e-5       # CFAR cells with |x - T*avg| / (T*avg) < NEAR_TOL are "near-threshold"


def rel_err(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))


MAX_TOL = 1e-5        # max|RDM_gpu - RDM_ref| / max|RDM_ref|   (SURVEY.md §8d's second figure)


def max_rel(a, b):
    return float(np.max(np.abs(np.asarray(a, np.float64) - b)) / np.max(np.abs(b)))


def oracle_cfar_dict(spec_cfar):
    d = spec_cfar.as_dict()
    d["zero_v_div"] = spec_cfar.zero_v_div
    return d


def oracle_rdm(name, echo):
    """fp64 RDM of fun_MTD_produce for the preset, from the C oracle."""
    e = np.asarray(echo)
    P, R = e.shape[-2], e.shape[-1]
    return coracle.pc_mtd(e.astype(np.complex128), coracle.preset(name, P, R))


def oracle_flags(rdm, cfar_obj, near_tol=NEAR_TOL):
    """(flag, flagV, ambiguous) from the loop-faithful numpy executeCFAR chain."""
    c = oracle_cfar_dict(cfar_obj)
    segs1 = [(a + 1, b) for a, b in cfar_obj.segments] or [(1, rdm.shape[-1])]
    out = [ref.main_cfar_chain(r, c, segs1, cfar_obj.zero_v_div, near_tol=near_tol) for r in rdm]
    return (np.stack([o[0] for o in out]).astype(np.uint8), np.stack([o[1] for o in out]).astype(np.uint8),
            np.stack([o[2] for o in out]))


def oracle_flags_c(rdm, cfar_obj, near_tol=NEAR_TOL):
    """oracle_flags from the C restatement (same rules, incl. the near-threshold mask;
    cross-checked against the numpy oracle in test_oracle.py) for large shapes."""
    c = oracle_cfar_dict(cfar_obj)
    segs0 = list(cfar_obj.segments) or [(0, rdm.shape[-1])]
    return coracle.cfar(rdm, c, segs0, near_tol=near_tol)


def flag_mismatch(gpu, want, amb):
    """(hard mismatches outside the ambiguity band, mismatches inside it)."""
    diff = np.asarray(gpu) != np.asarray(want)
    return int((diff & ~amb).sum()), int((diff & amb).sum())

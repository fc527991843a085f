#!/usr/bin/env python3
"""The MEX drop-ins at MATLAB's call granularity: each shim of
radar-signal-process_amd/mex linked with the fake MEX runtime (tests/mex_stub, built by
__graft_entry__.build()) and called as MATLAB calls it --

  * fun_MTD_produce(echoData, params): ONE CPI per call, a complex double P x R column-major
    echo in, a fresh P x R double RDM out (MTD/main_produce_dataset_win_xzr_v2.m:136);
  * executeCFAR(rdm, ...): one call per column segment of fun_CFARflag
    (CFAR_WangCai/main_cfar.m:147-154), a double V x R' segment in, fresh double flag / flagV out.

The shim allocates its outputs with mxCreateDoubleMatrix on every call (fresh, zeroed pages, as
MATLAB's allocator hands them out), and the caller frees them after the call.  Inputs are created
once (MATLAB's own slicing is not the shim's cost).  With --compare, the round-4 shims
(lib*_mex_r4.so, built from commit f50fb2c's sources: float / byte outputs widened by a serial
loop in the shim) run interleaved with the current ones, and their outputs must be identical.

    python tools/mex_bench.py [--P 128 --R 4096] [--seconds 3] [--compare [--reps 3]] [--json out.json]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "mex_stub", "build")
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))


class Shim:
    def __init__(self, path):
        self.path = path
        self.lib = lib = C.CDLL(path)
        vp = C.c_void_p
        lib.rt_double.restype = vp
        lib.rt_double.argtypes = [C.c_size_t, C.c_size_t, vp, C.c_int]
        lib.rt_struct.restype = vp
        lib.rt_struct.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(vp)]
        lib.rt_free.argtypes = [vp]
        lib.rt_call.restype = C.c_int
        lib.rt_call.argtypes = [C.c_int, C.POINTER(vp), C.c_int, C.POINTER(vp)]
        lib.rt_data.restype = C.POINTER(C.c_double)
        lib.rt_data.argtypes = [vp]
        lib.rt_errmsg.restype = C.c_char_p

    def arg(self, x):
        if isinstance(x, dict):
            names = (C.c_char_p * len(x))(*[k.encode() for k in x])
            vals = (C.c_void_p * len(x))(*[self.arg(v) for v in x.values()])
            return self.lib.rt_struct(len(x), names, vals)
        a = np.atleast_2d(np.asarray(x))
        cplx = np.iscomplexobj(a)
        f = np.asfortranarray(a.astype(np.complex128 if cplx else np.float64))
        return self.lib.rt_double(a.shape[0], a.shape[1], f.ctypes.data, 1 if cplx else 0)

    def call(self, nlhs, prhs, keep=False):
        """prhs: prepared argument pointers (owned by the caller); returns output pointers
        (freed here unless keep)."""
        plhs = (C.c_void_p * max(1, nlhs))()
        args = (C.c_void_p * len(prhs))(*prhs)
        if self.lib.rt_call(nlhs, plhs, len(prhs), args):
            raise RuntimeError(self.lib.rt_errmsg().decode())
        out = [plhs[i] for i in range(nlhs)]
        if not keep:
            for p in out:
                self.lib.rt_free(p)
        return out

    def data(self, p, n):
        return np.ctypeslib.as_array(self.lib.rt_data(p), shape=(n,)).copy()


def rate(fn, seconds):
    fn()   # first call: context creation, pinned rings
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds and n >= 5:
            return n / dt, n


def v2_params(P, R):
    return {"prtNum": float(P), "fs": 25e6, "B": 20e6, "tao": np.array([[0.16e-6, 8e-6, 28e-6]]),
            "point_prt": np.array([[R, 228, 723, R - 951]], dtype=np.float64)}


def run(P=128, R=4096, seconds=3.0, compare=False, reps=1):
    """Each leg `reps` times, the shims alternating (current, r4, current, r4, ...), so drift of
    the box's state hits both; the median rate is reported."""
    from rsp import presets, synth
    spec = presets.v2(P, R)
    echoes = synth.echo_numpy(spec, 4, seed=31).astype(np.complex128)
    names = ["current"] + (["r4"] if compare else [])
    files = {"current": "lib%s_mex.so", "r4": "lib%s_mex_r4.so"}
    out = {"shape": [P, R], "seconds_per_leg": seconds, "reps": reps, "fun_MTD_produce": {}, "executeCFAR": {}}
    ref = {}
    mtd = {nm: Shim(os.path.join(BUILD, files[nm] % "fun_MTD_produce")) for nm in names}
    margs = {nm: [[sh.arg(e), sh.arg(v2_params(P, R))] for e in echoes] for nm, sh in mtd.items()}
    rates = {nm: [] for nm in names}
    for _ in range(reps):
        for nm in names:
            sh, args, i = mtd[nm], margs[nm], [0]

            def one():
                sh.call(1, args[i[0] % len(args)])
                i[0] += 1
            rates[nm].append(rate(one, seconds)[0])
    for nm in names:
        sh = mtd[nm]
        p = sh.call(1, margs[nm][0], keep=True)[0]
        ref.setdefault("mtd", {})[nm] = sh.data(p, P * R)
        sh.lib.rt_free(p)
        out["fun_MTD_produce"][nm] = {"calls_per_s": round(float(np.median(rates[nm])), 1),
                                      "runs": [round(r, 1) for r in rates[nm]]}
        for a in margs[nm]:
            for x in a:
                sh.lib.rt_free(x)
    # executeCFAR on the chain's own RDM, per fun_CFARflag segment (v2 CFAR segments) and whole
    rdm = ref["mtd"]["current"].reshape((P, R), order="F")
    cf = presets.default_cfar(spec)
    segs = [(a, b) for a, b in cf.segments]
    scal = [5, 7, cf.TR, 0, 5, 7, cf.TV, 0, cf.M0, 1]
    cfs = {nm: Shim(os.path.join(BUILD, files[nm] % "executeCFAR")) for nm in names}
    sargs = {nm: [[sh.arg(np.ascontiguousarray(rdm[:, a:b]))] + [sh.arg(float(v)) for v in scal] for a, b in segs]
             for nm, sh in cfs.items()}
    wargs = {nm: [sh.arg(rdm)] + [sh.arg(float(v)) for v in scal] for nm, sh in cfs.items()}
    fr = {nm: [] for nm in names}
    wr = {nm: [] for nm in names}
    for _ in range(reps):
        for nm in names:
            sh = cfs[nm]

            def frame():
                for a in sargs[nm]:
                    sh.call(2, a)
            fr[nm].append(rate(frame, seconds)[0])
            wr[nm].append(rate(lambda: sh.call(2, wargs[nm]), seconds)[0])
    for nm in names:
        sh = cfs[nm]
        f = sh.call(2, wargs[nm], keep=True)
        ref.setdefault("cfar", {})[nm] = np.concatenate([sh.data(p, P * R) for p in f])
        for p in f:
            sh.lib.rt_free(p)
        out["executeCFAR"][nm] = {"frames_per_s": round(float(np.median(fr[nm])), 1),
                                  "segment_calls_per_frame": len(segs),
                                  "whole_rdm_calls_per_s": round(float(np.median(wr[nm])), 1),
                                  "frame_runs": [round(r, 1) for r in fr[nm]]}
        for a in sargs[nm] + [wargs[nm]]:
            for x in a:
                sh.lib.rt_free(x)
    if compare:
        out["identical"] = bool(np.array_equal(ref["mtd"]["current"], ref["mtd"]["r4"]) and
                                np.array_equal(ref["cfar"]["current"], ref["cfar"]["r4"]))
        out["speedup_fun_MTD_produce"] = round(out["fun_MTD_produce"]["current"]["calls_per_s"] /
                                               out["fun_MTD_produce"]["r4"]["calls_per_s"], 3)
        out["speedup_executeCFAR_frame"] = round(out["executeCFAR"]["current"]["frames_per_s"] /
                                                 out["executeCFAR"]["r4"]["frames_per_s"], 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=128)
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--compare", action="store_true")
    ap.add_argument("--reps", type=int, default=1, help="legs per shim, alternating (median reported)")
    ap.add_argument("--json", default=None)
    ap.add_argument("--trace", action="store_true",
                    help="RSP_HOST_TRACE=1: the library prints a per-call phase breakdown on stderr")
    a = ap.parse_args()
    if a.trace:
        os.environ["RSP_HOST_TRACE"] = "1"
    out = run(a.P, a.R, a.seconds, a.compare, a.reps)
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where a host-API call with NEW output arrays spends its time: per call,
the numpy allocation of the three outputs, rsp_pc_mtd_cfar itself, and the release of the
outputs (the munmap of ~100 MB at 32 CPIs), for fresh arrays vs reused ones; c3 shape, MATLAB
column-major C128 echo.  Also the same with the library's output prefault off (RSP_PREFAULT=0
in a second process).

    python tools/host_fresh_probe.py [--batch 32] [--seconds 1.5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=1.5)
    a = ap.parse_args()
    from rsp import _capi as capi, presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec)
    n = a.batch
    echo = synth.echo_numpy(spec, n, seed=5).astype(np.complex128)
    h = np.ascontiguousarray(np.swapaxes(echo, 1, 2))
    V, Ro = eng.shape
    out = {"batch": n, "prefault": os.environ.get("RSP_PREFAULT", "1")}
    reused = (np.empty((n, Ro, V), np.float32), np.empty((n, Ro, V), np.uint8), np.empty((n, Ro, V), np.uint8))
    for mode in ("fresh", "reused"):
        ta = tc = tf = 0.0
        calls = 0
        t0 = time.perf_counter()
        while calls < 3 or time.perf_counter() - t0 < a.seconds:
            t1 = time.perf_counter()
            o = (np.empty((n, Ro, V), np.float32), np.empty((n, Ro, V), np.uint8),
                 np.empty((n, Ro, V), np.uint8)) if mode == "fresh" else reused
            t2 = time.perf_counter()
            eng.pc_mtd_cfar(h, cf, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR, out=o)
            t3 = time.perf_counter()
            if mode == "fresh":
                del o
            t4 = time.perf_counter()
            ta += t2 - t1
            tc += t3 - t2
            tf += t4 - t3
            calls += 1
        el = time.perf_counter() - t0
        out[mode] = {"cpi_per_s": round(n * calls / el, 1), "ms_per_call": round(el / calls * 1e3, 3),
                     "alloc_ms": round(ta / calls * 1e3, 3), "call_ms": round(tc / calls * 1e3, 3),
                     "free_ms": round(tf / calls * 1e3, 3), "calls": calls}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where the host-buffer path (rsp_pc_mtd_cfar with MATLAB's C128 column-major arrays) spends its
time: CPI/s at c3 for fresh output arrays (first-touch page faults, as a caller that allocates
per call pays them) against reused ones, over copy-thread counts and host chunk sizes, at 32
CPIs per call and at one."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))


def rate(eng, h, cf, capi, n, reuse, seconds=1.0):
    import numpy as np
    V, Ro = eng.shape
    out = None
    if reuse:
        out = (np.empty((n, Ro, V), np.float32), np.empty((n, Ro, V), np.uint8), np.empty((n, Ro, V), np.uint8))
    eng.pc_mtd_cfar(h, cf, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR, out=out)
    calls, t0 = 0, time.perf_counter()
    while calls < 3 or time.perf_counter() - t0 < seconds:
        eng.pc_mtd_cfar(h, cf, layout=capi.RSP_COLMAJOR, out_layout=capi.RSP_COLMAJOR, out=out)
        calls += 1
    return n * calls / (time.perf_counter() - t0)


def main():
    import numpy as np
    from rsp import _capi as capi
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    echo = synth.echo_numpy(spec, 32, seed=5).astype(np.complex128)
    h32 = np.ascontiguousarray(np.swapaxes(echo, 1, 2))
    h1 = np.ascontiguousarray(h32[:1])
    for threads in (1, 4, 8, 16):
        for chunk in (0, 1, 8):
            eng.set_host_pipeline(chunk, threads)
            r = [rate(eng, h32, cf, capi, 32, reuse) for reuse in (False, True)]
            print("threads %2d chunk %d  32/call: fresh %7.1f  reused %7.1f CPI/s" % (threads, chunk, r[0], r[1]),
                  flush=True)
        r = [rate(eng, h1, cf, capi, 1, reuse) for reuse in (False, True)]
        print("threads %2d          1/call: fresh %7.1f  reused %7.1f CPI/s" % (threads, r[0], r[1]), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

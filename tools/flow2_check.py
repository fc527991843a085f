#!/usr/bin/env python3
"""Round-6 A/B experiment check: the split persistent dataflow (RSP_FLOW2=n in
the environment; the library reads it once) against the chunked chain in a second process, bit
for bit, at c3 shapes (c64 and fp16, batches 1, 5, 19, 64, 1024) -- and the status word (a bounded
hand-off wait that expired) must stay 0.

    RSP_FLOW2=18 python tools/flow2_check.py > a.txt;  python tools/flow2_check.py > b.txt;  diff a.txt b.txt
"""
import ctypes as C
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))

import torch  # noqa: E402

from rsp import presets, synth  # noqa: E402
from rsp.engine import Engine  # noqa: E402


def digest(t):
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    lib = eng.lib
    have = hasattr(lib, "rsp_diag_flow2_status")
    for B, half, seed in ((1, False, 1), (5, False, 2), (19, True, 3), (64, False, 4), (1024, False, 5)):
        echo = synth.echo_torch(spec, B, seed=seed, device="cuda", half=half)
        rdm = torch.empty((B, 128, 4096), dtype=torch.float32, device="cuda")
        flag = torch.empty((B, 128, 4096), dtype=torch.uint8, device="cuda")
        fv = torch.empty((B, 128, 4096), dtype=torch.uint8, device="cuda")
        for rep in range(2):
            eng.run_dev(echo, rdm=rdm, flag=flag, flagV=fv, cfar=cf)
            torch.cuda.synchronize()
        st = C.c_int32(0)
        if have and os.environ.get("RSP_FLOW2"):
            lib.rsp_diag_flow2_status(eng.ctx, C.byref(st))
        print("B %d %s rdm %s flag %s flagV %s hits %d" % (B, "f16" if half else "c64", digest(rdm), digest(flag), digest(fv),
                                                         int(flag.sum())))
        print("status B %d: %d" % (B, st.value), file=sys.stderr)
        if st.value:
            sys.exit("a hand-off wait expired (B %d)" % B)
    eng.close()


if __name__ == "__main__":
    main()

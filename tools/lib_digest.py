#!/usr/bin/env python3
"""Bitwise digest of the chain's outputs for one library build (RSP_LIB selects it).

    RSP_LIB=radar-signal-process_amd/lib/ablate/librsp_X.so python tools/lib_digest.py > a.txt

Runs c3-, c4- and c5-shaped batches (GPU-drawn synthetic echo, fixed seeds) and prints one
sha256 per output plane set, so two builds that must be bit-identical (an instruction-
scheduling change, a hazard-padding change) can be compared with `diff`.
"""
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


def chain(P, R, B, half, seed):
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    echo = synth.echo_torch(spec, B, seed=seed, half=half)
    rdm = torch.empty((B, P, R), dtype=torch.float32, device="cuda")
    flag = torch.empty((B, P, R), dtype=torch.uint8, device="cuda")
    eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    print("v2 %dx%d B%d %s rdm %s flag %s hits %d" % (P, R, B, "f16" if half else "c64", digest(rdm),
                                                      digest(flag), int(flag.sum())))
    eng.close()


def window(P, R, F, win, seed):
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    frames = synth.echo_torch(spec, F + 1, seed=seed).reshape(1, F + 1, P, R)
    rdm = torch.empty((1, F, win, P, R), dtype=torch.float32, device="cuda")
    flag = torch.empty((1, F, win, P, R), dtype=torch.uint8, device="cuda")
    eng.window_dev(frames, win, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    print("win %dx%d F%d w%d rdm %s flag %s hits %d" % (P, R, F, win, digest(rdm), digest(flag), int(flag.sum())))
    eng.close()


if __name__ == "__main__":
    print("lib", os.environ.get("RSP_LIB", "default"))
    chain(128, 4096, 48, False, 11)
    chain(128, 4096, 8, True, 12)
    chain(64, 1024, 16, False, 13)
    chain(256, 8192, 4, False, 14)
    window(256, 8192, 4, 4, 15)
    window(256, 8192, 8, 4, 17)   # 64 MiB of flags in one chunk: the flag memset path (c4's)
    chain(512, 16384, 2, True, 16)

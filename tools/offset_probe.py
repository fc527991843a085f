#!/usr/bin/env python3
"""Address-placement probe: the same chain step with the echo placed at different byte offsets
inside a larger allocation (and the library's scratch re-allocated in between), to see
whether HBM channel placement moves the kernels' speed.
    python tools/offset_probe.py --config c4 --batch 32 --offsets 0 4096 65536 1048576"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "radar-signal-process_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--offsets", type=int, nargs="+", default=[0, 4096, 65536, 1 << 20, 3 << 20])
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    import torch
    import bench
    from rsp import presets, synth
    from rsp.engine import Engine
    c = dict(bench.CONFIGS[args.config])
    B = args.batch or c["batch"]
    spec = presets.make("v2", c["P"], c["R"])
    cfar = presets.default_cfar(spec)
    win = c["win"]
    eng = Engine(spec, device=0)
    nf = B + 1 if win else B
    base = synth.echo_torch(spec, nf, seed=5, device="cuda", half=c["half"])
    nbytes = base.numel() * base.element_size()
    P, R = spec.P, spec.R_out
    oshape = (1, B, win, P, R) if win else (B, P, R)
    rdm = torch.empty(oshape, dtype=torch.float32, device="cuda")
    flag = torch.empty(oshape, dtype=torch.uint8, device="cuda")
    big = torch.empty(nbytes + max(args.offsets) + 64, dtype=torch.uint8, device="cuda")
    for off in args.offsets + args.offsets[:1]:
        raw = big[off:off + nbytes]
        raw.copy_(base.view(torch.uint8).reshape(-1))
        echo = raw.view(base.dtype).reshape(base.shape)
        if win:
            echo = echo.reshape((1, nf) + tuple(base.shape[1:]))

        def step():
            if win:
                eng.window_dev(echo, win, rdm=rdm, flag=flag, cfar=cfar)
            else:
                eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cfar)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        units = B * (win or 1)
        print("offset %8d  %.4f ms/step  %.1f units/s" % (off, dt * 1e3, units / dt), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

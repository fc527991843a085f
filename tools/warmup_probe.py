#!/usr/bin/env python3
"""Per-step device time from the first step on (events around each step, no host sync in
between): how long the chain takes to reach its steady rate after start-up.
    python tools/warmup_probe.py --config c3 --steps 80"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "radar-signal-process_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=80)
    ap.add_argument("--pause-ms", type=float, default=0.0, help="host sleep before the run (idle GPU)")
    args = ap.parse_args()
    import time
    import torch
    import bench
    from rsp import presets, synth
    from rsp.engine import Engine
    c = dict(bench.CONFIGS[args.config])
    B, win = c["batch"], c["win"]
    spec = presets.make("v2", c["P"], c["R"])
    cfar = presets.default_cfar(spec) if c["cfar"] else None
    eng = Engine(spec, device=0)
    nf = B + 1 if win else B
    echo = synth.echo_torch(spec, nf, seed=5, device="cuda", half=c["half"])
    if win:
        echo = echo.reshape((1, nf) + tuple(echo.shape[1:]))
    P, R = spec.P, spec.R_out
    oshape = (1, B, win, P, R) if win else (B, P, R)
    rdm = torch.empty(oshape, dtype=torch.float32, device="cuda")
    flag = torch.empty(oshape, dtype=torch.uint8, device="cuda") if cfar else None

    def step():
        if win:
            eng.window_dev(echo, win, rdm=rdm, flag=flag, cfar=cfar)
        else:
            eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cfar)
    step()
    torch.cuda.synchronize()
    time.sleep(args.pause_ms / 1e3)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ev[0].record()
    for i in range(args.steps):
        step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    t = 0.0
    for i, m in enumerate(ms):
        t += m
        if i < 12 or i % 8 == 0 or i == len(ms) - 1:
            print("step %3d  t=%7.1f ms  %.4f ms" % (i, t, m), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Pulse-compression-only timing (rsp_pc_dev) for kernel experiments.

    RSP_LIB=... python tools/pc_bench.py [--P 128 --R 4096 --cpis 16 64 256 --iters 20 --chunk 0]

Prints us per CPI, rows/s and the PC kernel's own I/O rate (input read + output write).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=128)
    ap.add_argument("--R", type=int, default=4096)
    ap.add_argument("--preset", default="v2")
    ap.add_argument("--cpis", type=int, nargs="+", default=[16, 64, 256])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--chunk", type=int, default=0)
    args = ap.parse_args()
    import torch
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.make(args.preset, args.P, args.R)
    eng = Engine(spec, chunk=args.chunk)
    for n in args.cpis:
        echo = synth.echo_torch(spec, n, seed=5)
        out = torch.empty((n, spec.P, spec.R_out), dtype=torch.complex64, device="cuda")
        for _ in range(2):
            eng.pc_dev(echo, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            eng.pc_dev(echo, out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        io = n * spec.P * (spec.R * 8 + spec.R_out * 8)
        print("cpis %5d  %8.3f ms  %7.3f us/CPI  %6.2f Mrows/s  io %7.1f GB/s" % (
            n, ms, ms * 1e3 / n, n * spec.P / ms / 1e3, io / ms / 1e6), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

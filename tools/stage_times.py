#!/usr/bin/env python3
"""Standalone stage times at c3 shape (128 x 4096): PC alone, MTD alone (with and without the
CFAR), and the chained call, each over n CPIs on one stream with HIP events; prints us/CPI and
the stage's own HBM-side GB/s (PC: 8 MB/CPI, MTD: 4 + 2 (+0.5 flags) MB/CPI)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))


def timed(fn, reps=10):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3   # us per call


def main():
    import torch
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    P, R = 128, 4096
    mb = P * R * 8 / 1e6
    for n in [int(x) for x in os.environ.get("NS", "16 64 256").split()]:
        eng = Engine(spec, chunk=n, streams=1)
        echo = synth.echo_torch(spec, n, seed=3)
        pc = torch.empty((n, P, R), dtype=torch.complex64, device="cuda")
        rdm = torch.empty((n, P, R), dtype=torch.float32, device="cuda")
        flag = torch.empty((n, P, R), dtype=torch.uint8, device="cuda")
        t_pc = timed(lambda: eng.pc_dev(echo, pc))
        t_m = timed(lambda: eng.mtd_dev(pc, rdm=rdm))
        t_mc = timed(lambda: eng.mtd_dev(pc, rdm=rdm, flag=flag, cfar=cf))
        import dataclasses
        cf0 = dataclasses.replace(cf, rFlag=0)
        t_mv = timed(lambda: eng.mtd_dev(pc, rdm=rdm, flag=flag, cfar=cf0))
        t_all = timed(lambda: eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cf))
        print("n %4d | PC %.2f us/CPI (%.0f GB/s) | MTD %.2f (%.0f GB/s) | MTD+CFAR %.2f (%.0f GB/s) | "
              "MTD+CFARv %.2f | chain(1 stream) %.2f us/CPI" % (
                  n, t_pc / n, 2 * mb * n / t_pc * 1e3, t_m / n, 1.5 * mb * n / t_m * 1e3,
                  t_mc / n, 1.5625 * mb * n / t_mc * 1e3, t_mv / n, t_all / n), flush=True)
        eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Does the PC scratch round trip benefit from the Infinity Cache?  Times the MTD(+CFAR) stage
on a pulse-compressed buffer just written by PC ("hot") against the same buffer after a 1 GiB
fill has evicted it ("cold").  Single stream, events around the MTD call only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))


def main():
    import torch
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    flush = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    for n in (4, 16):
        eng = Engine(spec, chunk=n, streams=1)
        echo = synth.echo_torch(spec, n, seed=3)
        pc = torch.empty((n, 128, 4096), dtype=torch.complex64, device="cuda")
        rdm = torch.empty((n, 128, 4096), dtype=torch.float32, device="cuda")
        flag = torch.empty((n, 128, 4096), dtype=torch.uint8, device="cuda")
        res = {}
        for mode in ("hot", "cold", "hot", "cold"):
            tot = 0.0
            for _ in range(10):
                eng.pc_dev(echo, pc)
                if mode == "cold":
                    flush.fill_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                eng.mtd_dev(pc, rdm=rdm, flag=flag, cfar=cf)
                e1.record()
                torch.cuda.synchronize()
                tot += e0.elapsed_time(e1)
            res[mode] = tot / 10
        print("cpis %3d  mtd+cfar hot %.1f us  cold %.1f us  (%.1f vs %.1f us/CPI)" % (
            n, res["hot"] * 1e3, res["cold"] * 1e3, res["hot"] * 1e3 / n, res["cold"] * 1e3 / n), flush=True)
        eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Does the PC scratch round trip benefit from the Infinity Cache?  Times the MTD(+CFAR) stage
on a pulse-compressed buffer just written by PC ("hot") against the same buffer after a 1 GiB
fill has evicted it ("cold"), and -- the chain's own case (round 4) -- after one other chunk's
PC and MTD ran in between ("inter": what the second stream pipeline does between a chunk's PC and
its MTD at c3: 64 MiB of echo read, 64 MiB of scratch written and re-read, 40 MiB of RDM and
flags written).  Single stream, events around the
MTD call only.  The position of "inter" between "hot" and "cold" estimates the share of the
scratch reads the chain serves from HBM rather than from the Infinity Cache."""
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
        echo2 = synth.echo_torch(spec, n, seed=4)
        pc = torch.empty((n, 128, 4096), dtype=torch.complex64, device="cuda")
        pc2 = torch.empty((n, 128, 4096), dtype=torch.complex64, device="cuda")
        rdm = torch.empty((n, 128, 4096), dtype=torch.float32, device="cuda")
        flag = torch.empty((n, 128, 4096), dtype=torch.uint8, device="cuda")
        rdm2, flag2 = torch.empty_like(rdm), torch.empty_like(flag)
        res = {}
        for mode in ("hot", "cold", "inter", "hot", "cold", "inter"):
            tot = 0.0
            for _ in range(10):
                eng.pc_dev(echo, pc)
                if mode == "cold":
                    flush.fill_(1.0)
                elif mode == "inter":
                    eng.pc_dev(echo2, pc2)
                    eng.mtd_dev(pc2, rdm=rdm2, flag=flag2, cfar=cf)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                eng.mtd_dev(pc, rdm=rdm, flag=flag, cfar=cf)
                e1.record()
                torch.cuda.synchronize()
                tot += e0.elapsed_time(e1)
            res[mode] = tot / 10
        share = (res["inter"] - res["hot"]) / max(res["cold"] - res["hot"], 1e-9)
        print("cpis %3d  mtd+cfar hot %.1f us  inter %.1f us  cold %.1f us  (%.2f / %.2f / %.2f us/CPI); "
              "estimated HBM-served share of the chain's scratch reads %.2f" % (
                  n, res["hot"] * 1e3, res["inter"] * 1e3, res["cold"] * 1e3, res["hot"] * 1e3 / n,
                  res["inter"] * 1e3 / n, res["cold"] * 1e3 / n, share), flush=True)
        eng.close()


if __name__ == "__main__":
    main()

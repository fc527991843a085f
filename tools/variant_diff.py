#!/usr/bin/env python3
"""Localise where a library variant's pulse-compression / MTD output departs from the base build.

    python tools/variant_diff.py base dma2 mdma      (libraries radar-signal-process_amd/lib/ablate/librsp_<v>.so)

Each variant runs in its own process (RSP_LIB) on the same c3-shaped batch (16 CPIs, GPU-drawn
echo) and saves PC rows and the RDM; the first variant is the reference.  Prints, per variant,
the differing PC rows (count, first few, max |diff|) and RDM cells."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = "/tmp/rsp_vdiff"   # (64 MB per plane: kept out of gpurun_out, which travels back)


def run_one(name):
    os.makedirs(OUT, exist_ok=True)
    sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))
    import numpy as np
    import torch
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    echo = synth.echo_torch(spec, 16, seed=21)
    pc = torch.empty((16, 128, 4096), dtype=torch.complex64, device="cuda")
    eng.pc_dev(echo, pc)
    rdm = torch.empty((16, 128, 4096), dtype=torch.float32, device="cuda")
    flag = torch.empty((16, 128, 4096), dtype=torch.uint8, device="cuda")
    eng.mtd_dev(pc, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    np.save(os.path.join(OUT, "vdiff_pc_%s.npy" % name), pc.cpu().numpy())
    np.save(os.path.join(OUT, "vdiff_rdm_%s.npy" % name), rdm.cpu().numpy())


def main():
    names = sys.argv[1:]
    if os.environ.get("VDIFF_ONE"):
        return run_one(os.environ["VDIFF_ONE"])
    for n in names:
        env = dict(os.environ, VDIFF_ONE=n, RSP_LIB=os.path.join(ROOT, "radar-signal-process_amd", "lib", "ablate",
                                                                  "librsp_%s.so" % n))
        subprocess.check_call([sys.executable, os.path.abspath(__file__)], env=env, timeout=120)
    import numpy as np
    ref_pc = np.load(os.path.join(OUT, "vdiff_pc_%s.npy" % names[0])).reshape(-1, 4096)
    ref_rdm = np.load(os.path.join(OUT, "vdiff_rdm_%s.npy" % names[0])).reshape(-1, 4096)
    for n in names[1:]:
        pc = np.load(os.path.join(OUT, "vdiff_pc_%s.npy" % n)).reshape(-1, 4096)
        rdm = np.load(os.path.join(OUT, "vdiff_rdm_%s.npy" % n)).reshape(-1, 4096)
        d = np.abs(pc - ref_pc).max(axis=1)
        rows = np.nonzero(d > 0)[0]
        cols = np.nonzero(np.abs(pc - ref_pc).max(axis=0) > 0)[0]
        dr = np.abs(rdm - ref_rdm)
        print("%s: PC rows differing %d of %d (first %s), columns %s..%s, max |d| %.3g (ref max %.3g); "
              "RDM cells differing %d, max |d| %.3g" % (
                  n, len(rows), len(d), rows[:8].tolist(), cols[:1].tolist(), cols[-1:].tolist(), d.max(),
                  np.abs(ref_pc).max(), int((dr > 0).sum()), dr.max()), flush=True)


if __name__ == "__main__":
    main()

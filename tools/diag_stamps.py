#!/usr/bin/env python3
"""Per-phase time inside the PC and MTD kernels, from the dev-only stamped build
(tools/build_variant.sh stamps -DRSP_DIAG_STAMPS; RSP_LIB=.../librsp_stamps.so).

PC (rsp_pc_dev over --cpis CPIs, one launch per call): per workgroup, slot 0 entry, 1 the
row's loads arrived (waited), 2 FIR done, 3 forward FFT, 4 spectrum multiply, 5 inverse FFT,
6 stores issued, 7 stores done (waited).  MTD (rsp_mtd_cfar_dev, one pipeline, two chunks so
the second launch carries the first chunk's range stage): 0 entry, 1 loads + range gathers
arrived (waited), 2 FFT, 3 magnitude stored, 4 Doppler CFAR + hit list, 5 tile done, 6 range
job done, 7 tail hits + all stores done (waited).  Slots 8/9: 100 MHz clock at entry / exit.
A waited boundary ends overlap that the real kernel has, so read the phases as a breakdown,
not as the kernel's time.

Usage: RSP_LIB=... python tools/diag_stamps.py [--config c3|c5] [--cpis 16] [--json out.json]
(c5: 512 x 16384 fp16, the 16384-point segment as 5 overlap-save blocks of 4096, 16-bin MTD tiles;
c4: the c4 kernels -- 256-pulse MTD tiles of 16 bins, 8192-point rows as 3 blocks -- on plain
256 x 8192 CPIs instead of sliding windows)
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))
SLOTS = 16
PC_PHASES = ["load", "fir", "fft_fwd", "spectrum", "fft_inv", "store_issue", "store_done"]
MTD_PHASES = ["load+gather", "fft", "mag_store", "doppler_cfar", "tile_end", "range_job", "tail+drain"]


def read(lib, k, nwg):
    buf = np.zeros(nwg * SLOTS, dtype=np.uint64)
    rc = lib.rsp_diag_stamps(k, buf.ctypes.data_as(C.POINTER(C.c_uint64)), C.c_int64(buf.size))
    assert rc == 0, rc
    return buf.reshape(nwg, SLOTS).astype(np.int64)


def summarize(st, phases, sel):
    st = st[sel]
    d = np.diff(st[:, :8], axis=1)
    life_rt = (st[:, 9] - st[:, 8]) * 10.0                   # ns (100 MHz)
    t0 = st[:, 8].min()
    out = {"workgroups": int(st.shape[0]),
           "lifetime_us_median": round(float(np.median(life_rt)) / 1e3, 3),
           "span_us": round(float((st[:, 9].max() - t0) * 10.0) / 1e3, 3),
           "start_us_p50": round(float(np.median(st[:, 8] - t0) * 10.0) / 1e3, 3),
           "cycles_median": {p: int(np.median(d[:, i])) for i, p in enumerate(phases)},
           "cycles_mean": {p: int(np.mean(d[:, i])) for i, p in enumerate(phases)}}
    if phases is PC_PHASES and st[:, 12].any():   # FIR sub-phases (short rows)
        f = np.diff(st[:, [1, 10, 11, 12, 2]], axis=1)
        out["fir_split_median"] = {p: int(np.median(f[:, i])) for i, p in
                                   enumerate(["zero+stage", "taps_loop", "stores", "sync"])}
    tot = d.sum(axis=1)
    out["cycles_total_median"] = int(np.median(tot))
    out["share_of_cycles"] = {p: round(float(np.sum(d[:, i]) / np.sum(tot)), 3) for i, p in enumerate(phases)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpis", type=int, default=16)
    ap.add_argument("--config", default="c3", choices=["c3", "c4", "c5"])
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch
    from rsp import presets, synth
    from rsp.engine import Engine
    # (P, R, fp16 input, overlap-save blocks of the long segment, MTD tile width)
    P, R, half, nsub, W = {"c3": (128, 4096, False, 1, 32), "c4": (256, 8192, False, 3, 16),
                           "c5": (512, 16384, True, 5, 16)}[args.config]
    spec = presets.v2(P, R)
    cf = presets.default_cfar(spec)
    n = args.cpis
    eng = Engine(spec, chunk=n, streams=1)
    lib = eng.lib
    lib.rsp_diag_stamps.restype = C.c_int
    lib.rsp_diag_stamps.argtypes = [C.c_int, C.POINTER(C.c_uint64), C.c_int64]
    echo = synth.echo_torch(spec, 2 * n, seed=3, half=half)
    pc = torch.empty((2 * n, spec.P, spec.R_out), dtype=torch.complex64, device="cuda")
    for _ in range(3):
        eng.pc_dev(echo[:n], pc[:n])
    torch.cuda.synchronize()
    nlong = n * spec.P * nsub                # one 4096-point row (block) per workgroup
    nshort = (n * spec.P + 3) // 4           # 4 rows of the 1024-point segment per workgroup
    st = read(lib, 0, nlong + nshort)
    res = {"pc_long_rows": summarize(st, PC_PHASES, slice(0, nlong)),
           "pc_short_rows": summarize(st, PC_PHASES, slice(nlong, nlong + nshort))}
    eng.pc_dev(echo, pc)
    rdm = torch.empty((2 * n, spec.P, spec.R_out), dtype=torch.float32, device="cuda")
    flag = torch.empty((2 * n, spec.P, spec.R_out), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        eng.mtd_dev(pc, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    nm = n * ((spec.R_out + W - 1) // W)     # W-bin tiles
    st = read(lib, 1, nm)
    res["mtd_with_range_job"] = summarize(st, MTD_PHASES, slice(0, nm))
    print(json.dumps(res, indent=1))
    if args.json:
        json.dump(res, open(args.json, "w"), indent=1)
    eng.close()


if __name__ == "__main__":
    main()

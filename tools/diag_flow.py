#!/usr/bin/env python3
"""Where the persistent dataflow kernel's time goes (dev-only stamped build):

    tools/build_variant.sh diag "-DRSP_DIAG_FLOW"
    RSP_LIB=radar-signal-process_amd/lib/ablate/librsp_diag.so python tools/diag_flow.py --flow 1

Runs the c3 chain (128 x 4096, --batch CPIs, CFAR) once as a warm-up and once stamped, then
reads every workgroup's first items {kind, CPI, index, t0 claimed + decoded, t1 waits done,
t2 published} (100 MHz clock) and prints, per item kind, the median / mean wait, body and the
gap to the workgroup's next item, the launch span, and how many items of each kind ran in
parallel on average.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))
WG, ITEMS = 1024, 512
KINDS = {1: "pc_long", 4: "pc_short", 2: "mtd", 3: "range"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flow", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--half", action="store_true")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(128, 4096)
    cf = presets.default_cfar(spec)
    eng = Engine(spec, device=0)
    lib = eng.lib
    lib.rsp_diag_flow.restype = C.c_int
    lib.rsp_diag_flow.argtypes = [C.POINTER(C.c_uint64), C.c_int64]
    lib.rsp_diag_flow_clear.restype = C.c_int
    eng.set_flow(args.flow)
    B = args.batch
    echo = synth.echo_torch(spec, B, seed=11, half=args.half)
    rdm = torch.empty((B, spec.V, spec.R_out), dtype=torch.float32, device="cuda")
    flag = torch.empty((B, spec.V, spec.R_out), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    assert lib.rsp_diag_flow_clear() == 0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    eng.run_dev(echo, rdm=rdm, flag=flag, cfar=cf)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1)
    assert eng.flow_status() == 0
    buf = np.zeros(WG * ITEMS * 4, dtype=np.uint64)
    assert lib.rsp_diag_flow(buf.ctypes.data_as(C.POINTER(C.c_uint64)), C.c_int64(buf.size)) == 0
    d = buf.reshape(WG, ITEMS, 4)
    kind = (d[:, :, 0] & 15).astype(np.int64)
    idx = (d[:, :, 0] >> 36).astype(np.int64)
    kind = np.where((kind == 1) & (idx >= spec.P), 4, kind)   # PC units past the long rows: short-row groups
    j = ((d[:, :, 0] >> 4) & 0xffffffff).astype(np.int64)
    t0, t1, t2 = (d[:, :, 1].astype(np.int64), d[:, :, 2].astype(np.int64), d[:, :, 3].astype(np.int64))
    valid = (t0 > 0) & (t2 > 0)
    base = t0[valid].min()
    span = (t2[valid].max() - base) * 10e-3
    out = {"flow": args.flow, "batch": B, "event_ms": round(ms, 4), "span_us": round(float(span), 2),
           "items": int(valid.sum()), "kinds": {}}
    # gap to the workgroup's next item
    nxt = np.full_like(t0, -1)
    nxt[:, :-1] = t0[:, 1:]
    for k, name in KINDS.items():
        sel = valid & (kind == k)
        if not sel.any():
            continue
        waitv = (t1[sel] - t0[sel]) * 10e-3 if k != 3 else (t1[sel] - t0[sel]) * 10e-3
        body = (t2[sel] - t1[sel]) * 10e-3
        g = (nxt[sel] - t2[sel]) * 10e-3
        g = g[nxt[sel] > 0]
        busy = float(np.sum(t2[sel] - t0[sel]) * 10e-3)
        out["kinds"][name] = {
            "n": int(sel.sum()),
            "wait_us": {"median": round(float(np.median(waitv)), 3), "mean": round(float(np.mean(waitv)), 3),
                        "p90": round(float(np.percentile(waitv, 90)), 3)},
            "body_us": {"median": round(float(np.median(body)), 3), "mean": round(float(np.mean(body)), 3),
                        "p90": round(float(np.percentile(body, 90)), 3)},
            "gap_us_median": round(float(np.median(g)), 3) if g.size else None,
            "avg_in_flight": round(busy / span, 1),
        }
    # idle share: per workgroup, time between its first t0 and last t2 not inside an item
    per_wg_busy = np.where(valid, t2 - t0, 0).sum(axis=1) * 10e-3
    per_wg_life = (np.where(valid, t2, 0).max(axis=1) - np.where(valid, t0, np.iinfo(np.int64).max).min(axis=1)) * 10e-3
    ok = per_wg_life > 0
    out["wg_busy_share"] = round(float(per_wg_busy[ok].sum() / per_wg_life[ok].sum()), 4)
    out["cpi_per_s_event"] = round(B / (ms * 1e-3), 1)
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    eng.close()


if __name__ == "__main__":
    main()

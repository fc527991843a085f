#!/usr/bin/env python3
"""Generate tests/golden/ingest_*.npz: a small synthetic PRT record stream (the format of
FrameDataRead_xzr.m, written by oracle/ingest_ref.prt_record) with its fp64 oracle decode
(oracle/ingest_ref.FrameReader).  The reference ships no .bin capture and no DBF coefficient
file, so the inputs are synthetic (seeded) and the expected outputs come from the oracle:
these pin the oracle's behaviour over time and give the GPU path a fixed target.

Run from the repo root:  python tests/golden/make_golden_ingest.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle")]

import ingest_ref as ref  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def synth_frame(prt, point, ch, beams, seed, frame_no=0):
    """int16 I/Q records and a beam x channel DBF matrix (unit-modulus steering weights)."""
    rng = np.random.default_rng(seed)
    iq = rng.integers(-30000, 30000, size=(prt, point, ch, 2), dtype=np.int16)
    ang = rng.uniform(-np.pi, np.pi, size=(beams, ch))
    dbf = np.exp(1j * ang) * rng.uniform(0.5, 1.0, size=(beams, ch))
    servo = rng.integers(0, 3600, size=prt)
    cfg = dict(prtNum=prt, point_PRT=point, channel_num=ch, beam_num=beams, bytesFrameHead=64,
               bytesFrameEnd=64, bytesFrameRealtime=128)
    stream = b"".join(ref.prt_record(iq[p], frame_no=frame_no, pulse_no=p, servo=int(servo[p]), pulse_num=prt,
                                     timer=1000 * p, cfg=cfg) for p in range(prt))
    return iq, dbf, servo, cfg, stream


def synth_mixed_frame(types, point, ch, beams, seed, channel_num=None):
    """A frame whose PRT p carries data type types[p]: DDC (1) int16 I/Q, ADC (0) int16 per
    channel, or the 24-bit DBF layout (2) -- random bytes where the middle and high byte of a
    value are zero half the time each, so the uint8 arithmetic gives both saturated and plain
    values.  Returns (dbf, cfg, stream)."""
    rng = np.random.default_rng(seed)
    prt = len(types)
    cn = ch if channel_num is None else channel_num
    ang = rng.uniform(-np.pi, np.pi, size=(beams, cn))
    dbf = np.exp(1j * ang) * rng.uniform(0.5, 1.0, size=(beams, cn))
    cfg = dict(prtNum=prt, point_PRT=point, channel_num=cn, beam_num=beams, bytesFrameHead=64,
               bytesFrameEnd=64, bytesFrameRealtime=128)
    recs = []
    for p, t in enumerate(types):
        shape = np.zeros((point, ch), dtype=np.int8)
        if t == 1:
            iq = rng.integers(-30000, 30000, size=(point, ch, 2), dtype=np.int16)
            recs.append(ref.prt_record(iq, pulse_no=p, servo=p * 7, pulse_num=prt, cfg=cfg))
            continue
        if t == 0:
            pay = rng.integers(-32768, 32768, size=(point, ch), dtype=np.int16).astype("<i2").tobytes()
        else:
            L = 6 * ch + (8 - (6 * ch) % 8)
            b = rng.integers(0, 256, size=(point, L), dtype=np.uint8)
            keep = rng.random(size=(point, L)) < 0.5
            col = np.arange(L) % 3
            b[(col > 0)[None, :] & ~keep] = 0
            pay = b.tobytes()
        recs.append(ref.prt_record(shape, pulse_no=p, servo=p * 7, pulse_num=prt, cfg=cfg, data_type=t, payload=pay))
    return dbf, cfg, b"".join(recs)


def main():
    prt, point, ch, beams = 6, 40, 16, 13
    iq, dbf, servo, cfg, stream = synth_frame(prt, point, ch, beams, seed=2001)
    out, angles, done, end = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    assert done and not end
    np.savez_compressed(os.path.join(OUT, "ingest_6x40.npz"), stream=np.frombuffer(stream, dtype=np.uint8),
                        dbf=dbf, servo=angles, beams=out, cfg=np.array([prt, point, ch, beams]))
    print("wrote ingest_6x40.npz (%d bytes of records)" % len(stream))


if __name__ == "__main__":
    main()

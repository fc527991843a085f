"""GPU parity of the ingest path (rsp_ingest_frame_dev / rsp_ingest_ddc_dev through
rsp.ingest) against the fp64 oracle restatement of FrameDataRead_xzr.m (oracle/ingest_ref.py).

Bars: DDC beams rel-err <= 1e-6 (Frobenius, fp32 accumulation of int16 samples against
fp64); ADC and 24-bit DBF rows bit-exact (small integers); servo angles, per-PRT stop position
and the zero rows after it bit-exact; the frame flags (frameCompleted, is_global_stream_end)
equal.
"""
import os
import sys

import numpy as np
import pytest

import ingest_ref as ref

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_golden_ingest import synth_frame, synth_mixed_frame  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def ing():
    import torch
    assert torch.cuda.is_available()
    from rsp import ingest
    g = ingest.Ingest(0)
    yield g
    g.close()


def _rel(a, b):
    d = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (d if d else 1.0)


def _check(ing, stream, dbf, cfg):
    from rsp import ingest
    want, wang, wdone, wend = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    out, ang, done, end = ing.FrameDataRead_xzr(ingest.BytesStream(stream), dbf, cfg, 0)
    got = out.permute(1, 2, 0).cpu().numpy()           # MATLAB's prt x sample x beam
    assert (done, end) == (wdone, wend)
    np.testing.assert_array_equal(ang, wang)
    zero_rows = ~np.any(want != 0, axis=(1, 2))
    assert np.array_equal(~np.any(got != 0, axis=(1, 2)), zero_rows)
    assert _rel(got, want) < TOL, _rel(got, want)
    return got, done


def test_golden(ing):
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ingest_6x40.npz"))
    prt, point, ch, beams = (int(v) for v in g["cfg"])
    from rsp import ingest
    cfg = ingest.sig_config(prtNum=prt, point_PRT=point, channel_num=ch, beam_num=beams)
    out, ang, done, end = ing.FrameDataRead_xzr(ingest.BytesStream(g["stream"].tobytes()), g["dbf"], cfg, 0)
    assert done and not end
    assert _rel(out.permute(1, 2, 0).cpu().numpy(), g["beams"]) < TOL
    np.testing.assert_array_equal(ang, g["servo"])


@pytest.mark.parametrize("prt,point,ch", [(7, 3404, 16), (5, 1000, 16), (4, 257, 8), (3, 100, 3)])
def test_parity_shapes(ing, prt, point, ch):
    """The 16-channel specialisation (16-byte loads) and the generic channel loop."""
    iq, dbf, servo, cfg, stream = synth_frame(prt, point, ch, 13, seed=prt * 1000 + ch)
    _, done = _check(ing, stream, dbf, cfg)
    assert done


def test_v2_capture_frame(ing):
    """A full v2 capture frame: 332 PRTs x 3404 samples x 16 channels -> 13 beams."""
    iq, dbf, servo, cfg, stream = synth_frame(332, 3404, 16, 13, seed=99)
    _, done = _check(ing, stream, dbf, cfg)
    assert done


def test_bad_heads_and_truncation(ing):
    """Each of the reference's early returns stops the frame at the same PRT."""
    iq, dbf, servo, cfg, stream = synth_frame(8, 300, 16, 13, seed=5)
    rec = len(stream) // 8

    def patch(p, word, value):
        b = bytearray(stream)
        b[p * rec + 4 * word:p * rec + 4 * word + 4] = int(value).to_bytes(4, "little")
        return bytes(b)

    cases = [patch(2, 6, 0),                        # pulse_data_num = 0
             patch(5, 6, 299),                      # wrong sample count: size check
             patch(1, 7, 0 | (8 << 8)),             # data_type 0 (ADC)
             patch(6, 7, 2 | (8 << 8)),             # data_type 2 (DBF payload)
             stream[:3 * rec + 70],                 # cut inside PRT 3's realtime block
             stream[:6 * rec + 64 + 128 + 5000],    # cut inside PRT 6's payload
             stream[:8 * rec - 1],                  # PRT 7's tail cut: PRT 7 is stored
             b""]
    for s in cases:
        _check(ing, s, dbf, cfg)
    # a head with another channel count: MATLAB stops with an error in the DBF product
    # (:158, inner dimensions); the GPU path reports RSP_PRT_BAD_SHAPE and stops the frame
    from rsp import _capi, ingest
    bad = patch(4, 3, 15)
    with pytest.raises(ValueError):
        ref.FrameReader().read(ref.BytesStream(bad), dbf, cfg, 0)
    full, _, _, _ = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    import torch
    d = torch.frombuffer(bytearray(bad), dtype=torch.uint8).cuda()
    out, _, status = ing.decode_dev(d, len(bad), cfg, ing.dbf_device(dbf))
    st = status.cpu().numpy()
    assert st[4] == _capi.RSP_PRT_BAD_SHAPE and st[8] == 4
    got = out.permute(1, 2, 0).cpu().numpy()
    assert not got[4:].any() and _rel(got[:4], full[:4]) < TOL


def test_files_and_window_placement(ing, tmp_path):
    """Frames read through rsp.ingest.FileStream across files (a record split over a file
    boundary, and a read ending exactly at EOF, which skips a file as the reference does),
    and decoded straight into a [beam][frames][P][R] window buffer via beam_stride."""
    import torch
    from rsp import ingest
    iq0, dbf, _, cfg, s0 = synth_frame(4, 500, 16, 13, seed=11, frame_no=0)
    _, _, _, _, s1 = synth_frame(4, 500, 16, 13, seed=12, frame_no=1)
    rec = len(s0) // 4
    data = s0 + s1
    cut1 = rec + 100                 # PRT 1's realtime block straddles files 1 and 2
    cut2 = 5 * rec + 64              # file 2 ends exactly after PRT 5's head
    for i, c in enumerate([data[:cut1], data[cut1:cut2], b"\x00" * 77, data[cut2:]]):
        with open(ingest.DataFullPathGen(str(tmp_path), i + 1), "wb") as f:
            f.write(c)
    fs, ofs = ingest.FileStream(str(tmp_path)), ref.ContinuousFileStream(str(tmp_path))
    rd = ref.FrameReader()
    for frame in range(2):
        want, wang, wdone, wend = rd.read(ofs, dbf, cfg, frame)
        out, ang, done, end = ing.FrameDataRead_xzr(fs, dbf, cfg, frame)
        assert (done, end) == (wdone, wend) and done
        assert _rel(out.permute(1, 2, 0).cpu().numpy(), want) < TOL
    fs.close()
    # beam_stride: frame f of beam b at win[b, f]
    P, R, B = 4, 500, 13
    win = torch.zeros((B, 2, P, R), dtype=torch.complex64, device="cuda")
    d_dbf = ing.dbf_device(dbf)
    for f, s in enumerate((s0, s1)):
        d = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
        ing.decode_dev(d, len(s), cfg, d_dbf, out=win[:, f], beam_stride=2 * P * R)
    torch.cuda.synchronize()
    for f, s in enumerate((s0, s1)):
        want, _, _, _ = ref.FrameReader().read(ref.BytesStream(s), dbf, cfg, 0)
        assert _rel(win[:, f].permute(1, 2, 0).cpu().numpy(), want) < TOL


def _exact_rows(got, want, types):
    for p, t in enumerate(types):
        if t != 1:
            np.testing.assert_array_equal(got[p], want[p])


def test_adc_frame(ing):
    """ADC records (FrameDataRead_xzr.m:144-147): with channel_num == beam_num the int16
    matrix is the frame's beams, bit-exact."""
    types = [0] * 6
    dbf, cfg, stream = synth_mixed_frame(types, 3404, 13, 13, seed=21)
    got, done = _check(ing, stream, dbf, cfg)
    assert done
    want, _, _, _ = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    _exact_rows(got, want, types)


@pytest.mark.parametrize("ch,beams", [(16, 17), (13, 13), (4, 5)])
def test_dbf24_frame(ing, ch, beams):
    """The 24-bit DBF branch as MATLAB's uint8 arithmetic evaluates it, bit-exact."""
    types = [2] * 5
    dbf, cfg, stream = synth_mixed_frame(types, 1000, ch, beams, seed=ch)
    got, done = _check(ing, stream, dbf, cfg)
    assert done
    want, _, _, _ = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    _exact_rows(got, want, types)


def test_mixed_frame_and_cuts(ing):
    """A frame of DDC, ADC and DBF records (9 channels and 9 beams pass all three size checks):
    records are located by walking the heads from the first one whose size differs, and cuts
    inside each kind of record stop the frame where the reference stops."""
    types = [1, 1, 0, 2, 3, 2, 1, 0, 1, 2, 255, 1, 1, 1]
    dbf, cfg, stream = synth_mixed_frame(types, 3404, 9, 9, seed=33)
    got, done = _check(ing, stream, dbf, cfg)
    assert done
    want, _, _, _ = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    _exact_rows(got, want, types)
    offs = [0]
    for t in types:
        offs.append(offs[-1] + 192 + ref.payload_bytes(t, 3404, 9) + 64)
    for p in (2, 3, 4, 7, 10):   # inside the payload, then inside the tail
        _check(ing, stream[:offs[p] + 192 + 1000], dbf, cfg)
        _check(ing, stream[:offs[p + 1] - 10], dbf, cfg)


@pytest.mark.parametrize("seed", [1, 2])
def test_long_mixed_frame_walk(ing, seed):
    """A long frame of randomly mixed record kinds (three record sizes, runs of equal sizes and
    alternations): the wave's head walk resolves many records per round of candidate loads and
    must land on every record exactly as the serial walk does."""
    rng = np.random.default_rng(seed)
    types = [int(t) for t in rng.choice([0, 1, 2, 3], size=150, p=[0.3, 0.4, 0.2, 0.1])]
    types[:3] = [1, 1, 1]   # a speculative prefix, then the walk
    types[40:70] = [0] * 30  # a long run of one size inside the walk
    dbf, cfg, stream = synth_mixed_frame(types, 100, 9, 9, seed=40 + seed)
    got, done = _check(ing, stream, dbf, cfg)
    assert done
    want, _, _, _ = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    _exact_rows(got, want, types)


def test_dbf24_size_error_and_ddc_only(ing):
    """14 channels give an odd 24-bit value count: a MATLAB size error in the reference,
    RSP_PRT_BAD_SHAPE here; rsp_ingest_ddc_dev refuses the first non-DDC record."""
    import torch
    from rsp import _capi
    dbf, cfg, stream = synth_mixed_frame([1, 2, 1], 100, 14, 7, seed=3)
    with pytest.raises(ValueError):
        ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    d = torch.frombuffer(bytearray(stream), dtype=torch.uint8).cuda()
    out, _, status = ing.decode_dev(d, len(stream), cfg, ing.dbf_device(dbf))
    st = status.cpu().numpy()
    assert st[0] == _capi.RSP_PRT_OK and st[1] == _capi.RSP_PRT_BAD_SHAPE and st[3] == 1
    assert not out[:, 1:].any().item() and out[:, 0].abs().sum().item() > 0
    types = [1, 1, 0, 1]
    dbf, cfg, stream = synth_mixed_frame(types, 100, 9, 9, seed=4)
    d = torch.frombuffer(bytearray(stream), dtype=torch.uint8).cuda()
    _, _, status = ing.decode_dev(d, len(stream), cfg, ing.dbf_device(dbf), ddc_only=True)
    st = status.cpu().numpy()
    assert st[2] == _capi.RSP_PRT_UNSUPPORTED_TYPE and st[4] == 2


def test_unknown_type_records_are_zero_rows(ing):
    """Data types 3..255 (FrameDataRead_xzr.m:110-112 sizes the payload as DBF, :141 only
    typecasts it, :160-165 has no case): the row stays zeros(point_PRT, beam_num), passes the
    :171 size check whatever the head's channel and sample counts, and the frame goes on."""
    import torch
    from rsp import _capi
    dbf, cfg, stream = synth_mixed_frame([1, 1, 1], 200, 9, 9, seed=5)
    rec = len(stream) // 3
    odd = ref.prt_record(np.zeros((150, 5), np.int8), pulse_no=1, servo=99, pulse_num=4, cfg=cfg, data_type=7,
                         payload=bytes(range(256)) * 4)
    stream = stream[:rec] + odd + stream[rec:]
    cfg = dict(cfg, prtNum=4)
    want, ang, done, _ = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    assert done and not want[1].any() and ang[1] == 99
    d = torch.frombuffer(bytearray(stream), dtype=torch.uint8).cuda()
    out, servo, status = ing.decode_dev(d, len(stream), cfg, ing.dbf_device(dbf))
    st = status.cpu().numpy()
    assert (st[:4] == _capi.RSP_PRT_OK).all() and st[4] == 4
    got = out.cpu().numpy().transpose(1, 2, 0)
    assert not got[1].any() and int(servo[1].item()) == 99
    for p in (0, 2, 3):
        err = np.linalg.norm(got[p] - want[p]) / np.linalg.norm(want[p])
        assert err < 1e-6, (p, err)

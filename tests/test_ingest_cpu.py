"""Raw-data ingest on the CPU side: the oracle restatement of
FrameDataRead_xzr.m / read_continuous_file_stream.m against independent arithmetic and the
committed golden stream, the product's host-side file stream against the oracle's (the
EOF-exact file skip included), and the C ABI's record size."""
import os
import sys

import numpy as np
import pytest

import ingest_ref as ref

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_golden_ingest import synth_frame, synth_mixed_frame  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ingest_6x40.npz")


def test_oracle_decode_matches_direct_dbf():
    """The record parse + DBF equals an independent einsum of the int16 samples."""
    iq, dbf, servo, cfg, stream = synth_frame(5, 37, 16, 13, seed=7)
    out, angles, done, end = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    assert done and not end
    x = iq[..., 0].astype(np.float64) + 1j * iq[..., 1].astype(np.float64)     # [prt][s][ch]
    want = np.einsum("psc,bc->psb", x, dbf)
    np.testing.assert_allclose(out, want, rtol=0, atol=1e-9 * np.abs(want).max())
    np.testing.assert_array_equal(angles, servo)


def test_oracle_golden():
    g = np.load(GOLDEN)
    prt, point, ch, beams = (int(v) for v in g["cfg"])
    cfg = dict(prtNum=prt, point_PRT=point, channel_num=ch, beam_num=beams, bytesFrameHead=64,
               bytesFrameEnd=64, bytesFrameRealtime=128)
    out, angles, done, end = ref.FrameReader().read(ref.BytesStream(g["stream"].tobytes()), g["dbf"], cfg, 0)
    assert done and not end
    np.testing.assert_array_equal(out, g["beams"])
    np.testing.assert_array_equal(angles, g["servo"])


def test_oracle_early_returns():
    """A bad head or a short stream ends the frame at that PRT with the rest zero
    (FrameDataRead_xzr.m:62-67,90-94,171-176)."""
    iq, dbf, servo, cfg, stream = synth_frame(6, 40, 16, 13, seed=8)
    rec = len(stream) // 6
    full, _, _, _ = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    bad = bytearray(stream)
    bad[3 * rec + 6 * 4:3 * rec + 7 * 4] = (0).to_bytes(4, "little")          # pulse_data_num = 0 at PRT 3
    out, angles, done, end = ref.FrameReader().read(ref.BytesStream(bytes(bad)), dbf, cfg, 0)
    assert not done and end
    np.testing.assert_array_equal(out[:3], full[:3])
    assert not out[3:].any() and not angles[3:].any()
    out, _, done, end = ref.FrameReader().read(ref.BytesStream(stream[:4 * rec + 100]), dbf, cfg, 0)
    assert not done and end and not out[4:].any()
    np.testing.assert_array_equal(out[:4], full[:4])
    out, _, done, end = ref.FrameReader().read(ref.BytesStream(stream[:5 * rec - 10]), dbf, cfg, 0)   # tail cut
    assert not done and end
    np.testing.assert_array_equal(out[:5], full[:5])                               # PRT 4 was stored


def _write_files(tmp, chunks):
    for i, c in enumerate(chunks):
        with open(ref.data_full_path_gen(str(tmp), i + 1), "wb") as f:
            f.write(c)


@pytest.mark.parametrize("quirk_cut", [False, True])
def test_file_stream_matches_oracle(tmp_path, quirk_cut):
    """rsp.ingest.FileStream == oracle ContinuousFileStream over the same files and reads,
    including a read that ends exactly at a file's end (the reference then skips a file)."""
    from rsp import ingest
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, size=5000, dtype=np.uint8).tobytes()
    cuts = [0, 1000, 2200, 3000, 5000] if not quirk_cut else [0, 64, 1000, 1064, 5000]
    _write_files(tmp_path, [data[a:b] for a, b in zip(cuts, cuts[1:])])
    sizes = [64, 128, 700, 64] * 12
    a, b = ingest.FileStream(str(tmp_path)), ref.ContinuousFileStream(str(tmp_path))
    for n in sizes:
        ra, rb = a.read(n), b.read(n)
        assert ra == rb
        if ra[2]:
            break
    a.close()


def test_file_stream_skip_quirk(tmp_path):
    """read_continuous_file_stream.m:138-150 + :47-48: a read that ends exactly at EOF makes
    the next read open file k+2."""
    from rsp import ingest
    _write_files(tmp_path, [b"A" * 64, b"B" * 64, b"C" * 64])
    s = ingest.FileStream(str(tmp_path))
    assert s.read(64) == (b"A" * 64, 64, False)
    assert s.read(64)[0] == b"C" * 64
    s2 = ingest.FileStream(str(tmp_path), quirk=False)
    s2.read(64)
    assert s2.read(64)[0] == b"B" * 64


def test_dbf_coeff_text(tmp_path):
    """bin_to_mat_xzr.m:27-29: columns alternate I and Q per channel."""
    from rsp import ingest
    p = tmp_path / "coef.txt"
    p.write_text("1,2,3,4\n5 6 7 8\n")
    c = ingest.read_dbf_coeffs(str(p))
    np.testing.assert_array_equal(c, np.array([[1 + 2j, 3 + 4j], [5 + 6j, 7 + 8j]]))
    np.testing.assert_array_equal(ref.dbf_from_text([[1, 2, 3, 4], [5, 6, 7, 8]]), c)


def test_record_bytes_abi():
    """rsp_ingest_record_bytes: the v2 capture's 64 + 128 + 3404*16*4 + 64 bytes (no pad), and
    the 64-B padding of the payload (FrameDataRead_xzr.m:115-119)."""
    import ctypes as C
    from rsp import _capi, ingest
    lib = _capi.load_library()
    n = C.c_int64()
    assert lib.rsp_ingest_record_bytes(C.byref(ingest.Ingest.params(ingest.sig_config())), C.byref(n)) == 0
    assert n.value == 64 + 128 + 3404 * 16 * 4 + 64
    cfg = ingest.sig_config(point_PRT=37, channel_num=3)
    assert lib.rsp_ingest_record_bytes(C.byref(ingest.Ingest.params(cfg)), C.byref(n)) == 0
    assert n.value == 64 + 128 + ref.ddc_payload_bytes(37, 3) + 64 == 64 + 128 + 448 + 64
    bad = ingest.sig_config(point_PRT=0)
    assert lib.rsp_ingest_record_bytes(C.byref(ingest.Ingest.params(bad)), C.byref(n)) == _capi.RSP_ERR_ARG


def _direct_dbf24(raw, pdn, ch, beams):
    """The 24-bit branch's result written out directly: value j of a sample row is 255 when
    its middle or high byte is non-zero (uint8 saturation), else its low byte."""
    L = 6 * ch + (8 - (6 * ch) % 8)
    rows = np.frombuffer(raw[:pdn * L], dtype=np.uint8).reshape(pdn, L).astype(np.int64)
    v = np.where((rows[:, 1:3 * 2 * beams:3] | rows[:, 2:3 * 2 * beams:3]) != 0, 255, rows[:, 0:3 * 2 * beams:3])
    return v[:, 0::2] + 1j * v[:, 1::2]


@pytest.mark.parametrize("ch,beams", [(16, 17), (13, 13), (4, 5), (9, 9)])
def test_oracle_dbf24_literal(ch, beams):
    """FrameDataRead_xzr.m:130-135,162-164 with MATLAB's uint8 arithmetic: the oracle's
    column ranges and saturating sums equal the direct formulation, and the value count the
    product's size check uses (rsp.ingest.dbf24_values) is the oracle's column count."""
    from rsp import ingest
    dbf, cfg, stream = synth_mixed_frame([2, 2, 2], 23, ch, beams, seed=ch)
    assert ingest.dbf24_values(ch) == 2 * beams
    out, _, done, end = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    assert done and not end
    rec = len(stream) // 3
    for p in range(3):
        raw = stream[p * rec + 64 + 128:(p + 1) * rec - 64]
        np.testing.assert_array_equal(out[p], _direct_dbf24(raw, 23, ch, beams))
    vals = np.concatenate([out.real.ravel(), out.imag.ravel()])
    assert (vals == 255).any() and ((vals > 0) & (vals < 255)).any()


@pytest.mark.parametrize("ch", [2, 3, 6, 7, 14])
def test_oracle_dbf24_size_errors(ch):
    """Channel counts whose 24-bit rows give unequal column ranges or an odd value count are a
    MATLAB size error in the reference (the product reports RSP_PRT_BAD_SHAPE)."""
    from rsp import ingest
    assert ingest.dbf24_values(ch) == -1
    dbf, cfg, stream = synth_mixed_frame([2], 10, ch, 4, seed=ch)
    with pytest.raises(ValueError):
        ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)


def test_oracle_adc_and_mixed_frame():
    """ADC records are the int16 matrix itself (:144-147) and records of different types and
    sizes follow one another (each sized by its own head, :105-119)."""
    types = [1, 0, 2, 3, 2, 1, 0, 200, 1]
    dbf, cfg, stream = synth_mixed_frame(types, 31, 9, 9, seed=4)
    out, ang, done, end = ref.FrameReader().read(ref.BytesStream(stream), dbf, cfg, 0)
    assert done and not end
    off = 0
    for p, t in enumerate(types):
        size = ref.payload_bytes(t, 31, 9)
        raw = stream[off + 192:off + 192 + size]
        if t == 0:
            np.testing.assert_array_equal(out[p], np.frombuffer(raw[:31 * 9 * 2], "<i2").reshape(31, 9))
        elif t == 2:
            np.testing.assert_array_equal(out[p], _direct_dbf24(raw, 31, 9, 9))
        elif t > 2:   # no case at :160-165: the zeros(point_PRT, beam_num) row
            assert not out[p].any()
        off += 192 + size + 64
    assert off == len(stream)
    np.testing.assert_array_equal(ang, 7 * np.arange(len(types)))


def test_host_reader_stops_where_the_reference_does():
    """rsp.ingest.Ingest.read_frame_bytes reads exactly the bytes the oracle's reader consumes
    (a record sized by its head; no realtime block after pulse_data_num = 0; no tail after a
    failed size check), so the stream position after a frame matches."""
    from rsp import ingest
    types = [1, 0, 2, 1]
    dbf, cfg, stream = synth_mixed_frame(types, 20, 9, 9, seed=6)
    rec0 = 64 + 128 + ref.payload_bytes(1, 20, 9) + 64
    cases = {"full": stream, "cut": stream[:rec0 + 100]}
    b = bytearray(stream)
    b[rec0 + 12:rec0 + 16] = (5).to_bytes(4, "little")       # PRT 1 (ADC): 5 channels != 9 beams
    cases["shape"] = bytes(b)
    b = bytearray(stream)
    b[rec0 + 24:rec0 + 28] = (0).to_bytes(4, "little")       # PRT 1: pulse_data_num = 0
    cases["count"] = bytes(b)
    # a type-7 record whose 5 channels and 12 samples would fail every other type's size check:
    # no case at :160-165, so the reference keeps a zero row, reads the tail and goes on
    odd = ref.prt_record(np.zeros((12, 5), np.int8), pulse_no=1, pulse_num=4, cfg=cfg, data_type=7,
                         payload=bytes(ref.payload_bytes(7, 12, 5)))
    cases["type7"] = stream[:rec0] + odd + stream[rec0:]
    for name, s in cases.items():
        host, oracle = ingest.BytesStream(s), ref.BytesStream(s)
        data, ended = ingest.Ingest.read_frame_bytes(host, cfg)
        _, _, done, end = ref.FrameReader().read(oracle, dbf, cfg, 0)
        assert host._pos == oracle.pos == len(data), name
        assert ended == end, name
        if name == "type7":
            assert done and not end and len(data) == len(s) - rec0   # PRTs 1, 7, 0, 2: the last DDC record unread
